#!/bin/bash
# round 4, GPU call 22: the split target by rows (160 up to 24 rows, else 480): the step / search / end-to-end /
# concurrency / fp8 tests, then default bench lines with the stream latency lines, vs WMX_PACKED_TARGET=480
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04z8}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
if [ "${2:-}" != notest ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_step.py \
  tests/test_gpu_e2e.py tests/test_gpu_concurrent.py tests/test_gpu_mx8.py tests/test_gpu_align.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; fi
fi
for i in 1 2; do
  for t in 0 480; do
    E=""; if [ $t != 0 ]; then E="WMX_PACKED_TARGET=$t"; fi
    env $E timeout -k 10 400 python bench.py --steps 3 --no-cpu-baseline > $O/b${i}_t$t.json 2> $O/b${i}_t$t.err || { echo "bench failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_t$t.json'));m=d['decode_mode'];print('b${i}_t$t', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], [(s['model'], s['p50_ms']) for s in d['stream_latency']], d['stream_load']['p50_ms'])"
  done
done
exit 0
