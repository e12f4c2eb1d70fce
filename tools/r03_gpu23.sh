#!/bin/bash
# round 3 (session 2), GPU call 23: kernel trace of a short default bench: the word-alignment stage's kernels per queue
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zg}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
rm -rf /tmp/bprof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/bprof -o run -- python3 bench.py --steps 2 --warmup 1 \
  --no-cpu-baseline --no-stream > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
KT=$(find /tmp/bprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/stage_kernels.py "$KT" | tee $O/align_stage.txt
grep -o '"stage_ms": \[[^]]*\]' $O/bench.json
