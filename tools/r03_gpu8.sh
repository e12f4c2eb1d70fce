#!/bin/bash
# round 3, GPU call 8: PMC passes over the encoder attention kernel (4-wave and 8-wave forms), one pass per run
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_SCA"
for f in 4 8; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    WMX_ENC_ATTN=$f timeout -s KILL 90 rocprofv3 --kernel-include-regex enc_attn --pmc $P -d $O/f${f}_p$i -o pmc -- python3 tools/attn_pmc.py \
      > $O/f${f}_p$i.log 2>&1 || { echo "pmc pass f$f p$i failed"; tail -5 $O/f${f}_p$i.log; exit 1; }
  done
done
python tools/pmc_summary.py $O enc_attn | tee $O/summary.txt
find $O -name '*.csv' ! -name '*counter_collection.csv' -delete
