#!/bin/bash
# round 5, GPU call 12: the MX-fp8 128-deep ring without spills — MX-fp8 GPU tests, then the 16-window fp8
# translate line interleaved against the 64-deep MX build (WMX_LIB = libwmx_mx64.so), and an encoder layer breakdown
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05l}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_mx8.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  for v in k128 mx64; do
    if [ $v = mx64 ]; then export WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_mx64.so; else unset WMX_LIB; fi
    timeout -k 10 300 python bench.py --dtype fp8 --task translate --batch 16 --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_$v.json 2> $O/b${i}_$v.err || { echo "bench failed"; tail -5 $O/b${i}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_$v.json'));e=d['encoder'];g=e['isolated_gpu_batch'];print('b${i}_$v', d['value'], d['ms_per_step'], 'enc8', e['isolated_ms'], 'enc16', g['ms'], 'insitu', e['insitu_stage_ms'])"
  done
done
unset WMX_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/encprof.py float8 > $O/encprof.txt 2>&1 || { echo "encprof failed"; exit 1; }
f=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python tools/enc_layer_breakdown.py $f > $O/layer_float8.txt 2>&1; cat $O/layer_float8.txt; rm -f $f
exit 0
