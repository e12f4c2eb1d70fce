#!/bin/bash
# round 4, GPU call 6: the mixed decode step (WMX_DEC_MIXED=1) -- parity (test_gpu_step.py rerun), then interleaved
# default-line A/B at 8 windows and one 16-window pair
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04j}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 890 --timeout-method thread -m gpu tests/test_gpu_step.py \
  -k "mixed_step or folded_layernorm" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc)"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
run() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream "$@" \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag', d['value'], d['stage_ms'][5], r['layer_e2e_us'])"
}
run b8_base WMX_DEC_MIXED=0 --
run b8_mixed WMX_DEC_MIXED=1 --
run b8_base2 WMX_DEC_MIXED=0 --
run b8_mixed2 WMX_DEC_MIXED=1 --
run b16_base WMX_DEC_MIXED=0 -- --batch 16
run b16_mixed WMX_DEC_MIXED=1 -- --batch 16
exit 0
