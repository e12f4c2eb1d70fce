#!/bin/bash
# round 4, GPU call 29: stream_load with the due windows split over two in-step contexts (WhisperModel.groups = 2)
# vs one context; the e2e tests first
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zj}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_e2e.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; fi
for i in 1 2; do
  for g in 2 1; do
    WMX_STREAM_GROUPS=$g timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b${i}_g$g.json 2> $O/b${i}_g$g.err || { echo "bench failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_g$g.json'));l=d['stream_load'];print('b${i}_g$g', d['value'], l['p50_ms'], l['p90_ms'], l['windows_per_call'], l['tick_busy'], l.get('context_groups'))"
  done
done
exit 0
