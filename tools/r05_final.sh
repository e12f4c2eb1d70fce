#!/bin/bash
# round 5, final measurement pass (two calls: '<tag> tests' = the whole -m gpu suite + smoke; '<tag> bench' =
# the default bench line (with the CPU baseline),
# the f16 line, the MX-fp8 / bf16 encoder at 16 windows, and a rocprofv3 kernel-trace summary (the trace itself
# is deleted on the box: only the stats come back)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05z}
mkdir -p $O
export PYTHONUNBUFFERED=1
# the subprocess-rerun tests print nothing for minutes: a heartbeat file keeps the box's silence watchdog informed
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
# the suite in two calls (each under gpurun's 20-minute limit): 'tests1' = every file but test_gpu_step.py,
# 'tests2' = test_gpu_step.py + smoke
if [ "${2:-tests1}" = tests1 ]; then
  timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=25 -m gpu tests \
    --ignore=tests/test_gpu_step.py > $O/gputest1.log 2>&1
  rc=$?; tail -3 $O/gputest1.log
  if [ $rc -ne 0 ]; then echo "gpu tests failed (rc $rc): stopping"; exit 1; fi
  exit 0
fi
if [ "${2}" = tests2 ]; then
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=25 -m gpu \
    tests/test_gpu_step.py > $O/gputest2.log 2>&1
  rc=$?; tail -3 $O/gputest2.log
  if [ $rc -ne 0 ]; then echo "gpu tests failed (rc $rc): stopping"; exit 1; fi
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
  echo "tests + smoke ok"
  exit 0
fi
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; exit 1; }
head -c 300 $O/bench_default.json; echo
timeout -k 10 300 python bench.py --dtype f16 --steps 5 --no-cpu-baseline --no-stream > $O/bench_f16.json \
  2> $O/bench_f16.err || { echo f16 bench failed; exit 1; }
head -c 200 $O/bench_f16.json; echo
timeout -k 10 300 python bench.py --dtype fp8 --task translate --batch 16 --steps 3 --no-cpu-baseline --no-stream \
  > $O/bench_fp8_b16.json 2> $O/bench_fp8_b16.err || { echo fp8 bench failed; exit 1; }
timeout -k 10 300 python bench.py --batch 16 --steps 3 --no-cpu-baseline --no-stream > $O/bench_bf16_b16.json \
  2> $O/bench_bf16_b16.err || { echo bf16 b16 bench failed; exit 1; }
timeout -k 10 300 python bench.py --dtype int8 --steps 3 --no-cpu-baseline --no-stream > $O/bench_int8.json \
  2> $O/bench_int8.err || { echo int8 bench failed; exit 1; }
head -c 200 $O/bench_int8.json; echo
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 \
  --no-cpu-baseline --no-stream > $O/bench_prof.json 2> $O/bench_prof.err || { echo profiled bench failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 bench.py --dtype fp8 \
  --task translate --batch 16 --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/bench_prof_fp8.json \
  2> $O/bench_prof_fp8.err || { echo profiled fp8 bench failed; exit 1; }
for st in $(find $O/prof -name '*kernel_stats.csv'); do python tools/roofline_from_stats.py $st $O/bench_prof.json > $O/roofline_from_stats.json; done
for st in $(find $O/prof_fp8 -name '*kernel_stats.csv'); do python tools/roofline_from_stats.py $st $O/bench_prof_fp8.json > $O/roofline_from_stats_fp8.json; done
for st in $(find $O/prof -name '*kernel_stats.csv'); do python tools/roofline_from_stats.py $st $O/bench_default.json > $O/roofline_from_stats_vs_default.json; done
grep -h '"frac"\|agreement' $O/roofline_from_stats*.json
find $O/prof $O/prof_fp8 -name '*kernel_trace.csv' -delete
find $O/prof $O/prof_fp8 -name '*.db' -delete
du -sh $O
find $O/prof $O/prof_fp8 -type f
exit 0
