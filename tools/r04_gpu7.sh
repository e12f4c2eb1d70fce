#!/bin/bash
# round 4, GPU call 7: the mixed step with prefetched fold constants -- parity, then 4 interleaved 8-window pairs
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04l}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 890 --timeout-method thread -m gpu tests/test_gpu_step.py \
  -k "mixed_step" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc)"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
run() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream "$@" \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];e=r['layer_e2e_us'];print('$tag', d['value'], d['stage_ms'][5], round(sum(e.values()),1), e)"
}
for i in 1 2 3 4; do
  run b8_base$i WMX_DEC_MIXED=0 --
  run b8_mixed$i WMX_DEC_MIXED=1 --
done
exit 0
