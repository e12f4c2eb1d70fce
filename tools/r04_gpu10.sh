#!/bin/bash
# round 4, GPU call 10: alignment stage without per-layer head uploads / syncs and with pinned D2H -- the alignment
# and end-to-end tests, then three default bench lines (stage_ms[6] = the alignment stage)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04p}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_align.py \
  tests/test_gpu_e2e.py tests/test_gpu_concurrent.py tests/test_gpu_mx8.py -k "align or word or concurrent or e2e" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc)"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b8_$i.json 2> $O/b8_$i.err || { echo bench failed; exit 1; }
  python -c "import json;d=json.load(open('$O/b8_$i.json'));print('b8_$i', d['value'], d['stage_ms'])"
done
exit 0
