#!/bin/bash
# round 5, GPU call 9: the 64-deep half-tile ring as the gemm256 default — encoder parity (the whole-encoder tests at
# every depth, the LayerNorm fold, the conv front end, cross-K/V) and interleaved bench lines against the 32-deep
# ring (WMX_LIB = libwmx_bk32.so)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05i}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_wide.py tests/test_gpu_e2e.py tests/test_gpu_step.py -k "not beam_options and not folded_layernorm_step and not mixed_step and not fused_mlp and not separate_cross_q and not cross_records" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  for v in k64 bk32; do
    if [ $v = bk32 ]; then export WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_bk32.so; else unset WMX_LIB; fi
    timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_$v.json 2> $O/b${i}_$v.err || { echo "bench failed"; tail -5 $O/b${i}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_$v.json'));e=d['encoder'];g=e['isolated_gpu_batch'];print('b${i}_$v', d['value'], d['ms_per_step'], d['stage_ms'], 'enc4', e['isolated_ms'], 'enc8', g['ms'], g['mfma_util'], 'insitu', e['insitu_stage_ms'])"
  done
done
unset WMX_LIB
exit 0
