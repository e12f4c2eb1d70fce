#!/bin/bash
# round 4, GPU call 18: lockstep A/B on default bench lines (WMX_LOCKSTEP=1 default vs 0), interleaved, plus one
# phase probe without lockstep first (is this box slow-mode prone?)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04z2}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
if [ "${2:-}" = test ]; then
  timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_concurrent.py > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; grep "lone member" $O/tests.log
  if [ $rc -ne 0 ]; then echo "tests failed"; exit 1; fi
fi
for i in 1 2 3 4 5 6; do
  for ls in 0 1; do
    WMX_LOCKSTEP=$ls timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_ls$ls.json 2> $O/b${i}_ls$ls.err || { echo "bench failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_ls$ls.json'));m=d['decode_mode'];print('b${i}_ls$ls', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']])"
  done
done
exit 0
