#!/bin/bash
# round 5, GPU call 14: decoder self attention with the first K / V batch issued before the q / k / v stage — step /
# search / end-to-end GPU tests, then interleaved default bench lines against the build without (WMX_LIB)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05o}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_e2e.py \
  -k "not full_depth and not beam_options" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  for v in pre sa0; do
    if [ $v = sa0 ]; then export WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_sa0.so; else unset WMX_LIB; fi
    timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_$v.json 2> $O/b${i}_$v.err || { echo "bench failed"; tail -5 $O/b${i}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_$v.json'));r=d['roofline'];e=r.get('layer_e2e_us',{});print('b${i}_$v', d['value'], d['ms_per_step'], d['stage_ms'][5], r['frac'], e.get('self_attn'), d.get('self_attn_us'))"
  done
done
unset WMX_LIB
exit 0
