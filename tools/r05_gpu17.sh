#!/bin/bash
# round 5, GPU call 17: PMC summaries of the encoder pass on the half-tile rings ("with a PMC
# summary under profiles/"): matrix-pipe busy cycles and held clock per kernel (tools/mfma_util.py), and the HBM
# traffic of the pass (FETCH_SIZE / WRITE_SIZE in separate passes), bf16 and MX-fp8
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05s}
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for ct in bfloat16 float8; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mfma_$ct -o pmc --output-format csv -- python3 tools/encprof.py $ct > $O/mfma_$ct.log 2>&1
  rc=$?; echo "mfma $ct rc=$rc"; [ $rc -ne 0 ] && exit 1
  f=$(find $O/mfma_$ct -name '*counter_collection.csv' | head -1)
  python tools/mfma_util.py $f gemm256 gemm_mx8 enc_attn layernorm > $O/mfma_util_$ct.txt 2>&1; cat $O/mfma_util_$ct.txt
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d $O/${c}_$ct -o pmc --output-format csv -- python3 tools/encprof.py $ct > $O/${c}_$ct.log 2>&1
    rc=$?; echo "$c $ct rc=$rc"; [ $rc -ne 0 ] && exit 1
  done
done
find $O -name '*counter_collection.csv' | head -20
exit 0
