#!/bin/bash
# Round-6 GPU recipe (run on the GPU box from the repo root):  bash tools/r06_gpu.sh <tag> <what>
#   tests1  every -m gpu file but test_gpu_step.py
#   tests2  test_gpu_step.py + smoke
#   bench   the default bench line (CPU baseline and streaming lines included)
#   quick   the default bench line without the CPU baseline / streaming lines
#   k:<expr> one pytest -k selection over the whole -m gpu suite
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:?tag}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
# the subprocess-rerun tests print nothing for minutes: a heartbeat file keeps the box's silence watchdog informed
(while sleep 50; do date >> "$O/heartbeat.txt"; done) &
HB=$!
trap "kill $HB" EXIT
case "${2:-quick}" in
  tests1)
    timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=25 -m gpu tests \
      --ignore=tests/test_gpu_step.py > "$O/gputest1.log" 2>&1
    rc=$?; tail -3 "$O/gputest1.log"; exit $rc ;;
  tests2)
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread --durations=25 -m gpu \
      tests/test_gpu_step.py > "$O/gputest2.log" 2>&1
    rc=$?; tail -3 "$O/gputest2.log"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
    echo "tests + smoke ok" ;;
  k:*)
    timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests -k "${2#k:}" \
      > "$O/gputest_k.log" 2>&1
    rc=$?; tail -3 "$O/gputest_k.log"; exit $rc ;;
  bench)
    timeout -k 10 400 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { echo bench failed; exit 1; }
    head -c 400 "$O/bench_default.json"; echo ;;
  quick)
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-stream > "$O/bench_quick.json" 2> "$O/bench_quick.err" \
      || { echo bench failed; exit 1; }
    head -c 400 "$O/bench_quick.json"; echo ;;
esac
