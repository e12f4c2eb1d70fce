#!/bin/bash
# round 3 (session 2), GPU call 20: PMC passes over one 8-window bf16 encoder pass (real activations): held clock and
# MFMA-pipe busy per kernel kind, and the wave-cycle split
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zd}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
rm -rf /tmp/pmc1 /tmp/pmc2
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc1 -o run -- \
  python3 tools/encprof.py bfloat16 > $O/pmc1.log 2>&1 || { echo pmc1 failed; tail $O/pmc1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  --output-format csv -d /tmp/pmc2 -o run -- python3 tools/encprof.py bfloat16 > $O/pmc2.log 2>&1 || { echo pmc2 failed; exit 1; }
C1=$(find /tmp/pmc1 -name "*counter_collection.csv" -print -quit)
C2=$(find /tmp/pmc2 -name "*counter_collection.csv" -print -quit)
python3 tools/enc_pmc.py "$C1" "$C2" | tee $O/enc_pmc.txt
