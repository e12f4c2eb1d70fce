#!/bin/bash
# round 5, GPU call 7: the cross attention's chunk records merged by the cross out-projection (WMX_XATTN_RECSPLIT=1):
# bit-identity test, the step / search / concurrency tests with the switch set, interleaved bench lines on / off
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05g}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest -x -v -rP --timeout 250 --timeout-method thread -m gpu tests/test_gpu_step.py -k "bit_identical" > $O/tests_bit.log 2>&1
rc=$?; tail -2 $O/tests_bit.log
if [ $rc -ne 0 ]; then echo "bit test failed"; grep -E "FAILED|Error|assert|Mismatch" $O/tests_bit.log | head -20; exit 1; fi
WMX_XATTN_RECSPLIT=1 timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_concurrent.py -k "not folded_layernorm and not mixed_step and not fused_mlp and not separate_cross_q and not full_depth" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  for rs in 1 0; do
    WMX_XATTN_RECSPLIT=$rs timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_rs$rs.json 2> $O/b${i}_rs$rs.err || { echo "bench failed"; tail -5 $O/b${i}_rs$rs.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_rs$rs.json'));r=d['roofline'];e=r['layer_e2e_us'];print('b${i}_rs$rs', d['value'], d['ms_per_step'], d['stage_ms'][5], r['frac'], e['cross_attn'], e['dec_cross_out'])"
  done
done
exit 0
