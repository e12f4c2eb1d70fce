#!/bin/bash
# round 3 (session 2), GPU call 26: the MX-fp8 encoder pass: per-layer launch breakdown and a PMC pass (held clock,
# MFMA busy, wave-cycle split) per kernel kind
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zl}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
rm -rf /tmp/encprof /tmp/pmc1 /tmp/pmc2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py float8 \
  > $O/encprof.log 2>&1 || { echo encprof failed; exit 1; }
KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/enc_layer_breakdown.py "$KT" | tee $O/enc_layers_fp8.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc1 -o run -- \
  python3 tools/encprof.py float8 > $O/pmc1.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  --output-format csv -d /tmp/pmc2 -o run -- python3 tools/encprof.py float8 > $O/pmc2.log 2>&1 || { echo pmc2 failed; exit 1; }
C1=$(find /tmp/pmc1 -name "*counter_collection.csv" -print -quit)
C2=$(find /tmp/pmc2 -name "*counter_collection.csv" -print -quit)
python3 tools/enc_pmc.py "$C1" "$C2" | tee $O/enc_pmc_fp8.txt
