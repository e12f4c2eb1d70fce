#!/bin/bash
# round 5, GPU call 19: gemm256 with 8 row panels per column walk (WMX_G256_GM=8) — encoder tests, then interleaved
# default bench lines against the 4-panel build (WMX_LIB = libwmx_gm4.so)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05u}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_wide.py tests/test_gpu_step.py -k "full_depth or encoder or wide or greedy or fold or alignment" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  for v in gm8 gm4; do
    if [ $v = gm4 ]; then export WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_gm4.so; else unset WMX_LIB; fi
    timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_$v.json 2> $O/b${i}_$v.err || { echo "bench failed"; tail -5 $O/b${i}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_$v.json'));e=d['encoder'];g=e['isolated_gpu_batch'];print('b${i}_$v', d['value'], d['ms_per_step'], 'enc4', e['isolated_ms'], 'enc8', g['ms'], g['mfma_util'], 'insitu', e['insitu_stage_ms'], 'xkv', d['stage_ms'][2])"
  done
done
unset WMX_LIB
exit 0
