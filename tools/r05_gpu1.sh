#!/bin/bash
# round 5, GPU call 1: graph-branch microbenchmark; the concurrency / e2e tests on the lockstep-leave fix; the decode
# step's launches ablated one kind at a time (WMX_ABLATE, timing only) against default lines, interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05a}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 ./tools/mb_graph_fork > $O/mb_graph_fork.txt 2>&1 || { echo "mb failed"; cat $O/mb_graph_fork.txt; exit 1; }
cat $O/mb_graph_fork.txt
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_e2e.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; fi
for i in 1 2; do
  for ab in 0 4 2 1 8 16 6; do
    WMX_ABLATE=$ab timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_ab$ab.json 2> $O/b${i}_ab$ab.err || { echo "bench failed"; tail -5 $O/b${i}_ab$ab.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_ab$ab.json'));m=d['decode_mode'];print('b${i}_ab$ab', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], d['stage_ms'])"
  done
done
exit 0
