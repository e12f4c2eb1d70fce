#!/bin/bash
# round 4, GPU call 25: the 8-bit decode on the 80 KiB reduction budget -- fp8 tests, then the config-5 line twice
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zd}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_mx8.py tests/test_gpu_concurrent.py tests/test_gpu_rccl.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype fp8 --task translate --batch 16 --steps 3 --no-cpu-baseline --no-stream > $O/f8_$i.json 2> $O/f8_$i.err || { echo "bench failed"; exit 1; }
  python -c "import json;d=json.load(open('$O/f8_$i.json'));m=d['decode_mode'];print('f8_$i', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']])"
done
exit 0
