#!/bin/bash
# round 4, GPU call 9: kernel trace of a short default bench, reduced on the box to the alignment stage's anatomy
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04o}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/wmxprof -o run -- python3 bench.py --steps 2 \
  --warmup 1 --no-cpu-baseline --no-stream > $O/bench_prof.json 2> $O/bench_prof.err || { echo profiled bench failed; exit 1; }
T=$(find /tmp/wmxprof -name '*kernel_trace.csv' | head -1)
python tools/align_timeline.py $T > $O/align_timeline.txt 2>&1
python tools/stage_kernels.py $T > $O/stage_kernels.txt 2>&1
cat $O/align_timeline.txt | head -80
exit 0
