#!/bin/bash
# round 3 (session 2), GPU call 15: the rebuilt library: smoke, encoder pass timing (bf16 / MX-fp8), and a kernel
# trace of one isolated 8-window bf16 encoder pass broken down per layer launch
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03w}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python tools/enc_ab.py bfloat16 > $O/enc.txt 2>&1 || { echo enc failed; exit 1; }
timeout -k 10 200 python tools/enc_ab.py float8 >> $O/enc.txt 2>&1 || { echo enc8 failed; exit 1; }
cat $O/enc.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py bfloat16 \
  > $O/encprof.log 2>&1 || { echo encprof failed; exit 1; }
KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/enc_layer_breakdown.py "$KT" | tee $O/enc_layers.txt
