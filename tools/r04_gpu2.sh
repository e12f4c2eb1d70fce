#!/bin/bash
# round 4, GPU call 2: register-resident cross-K/V quantizer (parity), then fp8 / bf16 lines at 8 and 16 windows and
# the 16-window fp8 line with 4 context groups
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04e}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py \
  -k "alignment or forced_steps_wide" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc)"; grep -E "FAILED|Error" $O/tests.log | head -20; fi
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['value'], d['stage_ms'], d['decode_mode']['mode'] if d['decode_mode'] else None)"
}
run fp8_b16 --dtype fp8 --task translate --batch 16
run fp8_b16_g4 --dtype fp8 --task translate --batch 16 --groups 4
run fp8_b8 --dtype fp8 --batch 8
run bf16_b8 --batch 8
run bf16_b16 --batch 16
exit 0
