#!/bin/bash
# round 3, GPU call 4 (after the stream-K revert): the whole -m gpu suite, smoke, the default bench line (with the
# CPU baseline), an f16 line, and a rocprofv3 kernel-trace summary of a short bench run
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gputest.log 2>&1
rc=$?; tail -3 $O/gputest.log
if [ $rc -ne 0 ]; then echo "gpu tests failed (rc $rc): stopping"; exit 1; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; exit 1; }
head -c 400 $O/bench_default.json; echo
timeout -k 10 300 python bench.py --dtype f16 --steps 10 --warmup 2 --no-cpu-baseline --no-stream > $O/bench_f16.json 2> $O/bench_f16.err \
  || { echo f16 bench failed; exit 1; }
head -c 300 $O/bench_f16.json; echo
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline \
  --no-stream > $O/bench_prof.json 2> $O/bench_prof.err || { echo profiled bench failed; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -3
exit 0
