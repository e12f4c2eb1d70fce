#!/bin/bash
# round 4, GPU call 31: the per-chunk lockstep barrier (default now) vs the start barrier only (WMX_LOCKSTEP_CHUNKS=0):
# concurrency / e2e tests, then interleaved default bench lines
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zl}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_e2e.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep "lone member" $O/tests.log | head -2
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; fi
for i in 1 2 3 4; do
  for ch in 1 0; do
    WMX_LOCKSTEP_CHUNKS=$ch timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_ch$ch.json 2> $O/b${i}_ch$ch.err || { echo "bench failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_ch$ch.json'));m=d['decode_mode'];print('b${i}_ch$ch', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']])"
  done
done
exit 0
