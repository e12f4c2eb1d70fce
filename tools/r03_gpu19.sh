#!/bin/bash
# round 3 (session 2), GPU call 19: packed GELU + residual prefetch in the gemm256 epilogues: parity (encoder wide /
# full depth / small models, MX-fp8), then the encoder pass interleaved: pre-fold base, fold v2, current
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zb}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wide.py \
  tests/test_gpu_mx8.py tests/test_gpu_step.py -k "wide_encoder or encoder_layernorm_fold or small_models or mx8" > $O/tests.log 2>&1
rc=$?; grep -E "rel_l2|passed|failed|Error" $O/tests.log | tail -14
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3; do
  for v in base fold2 cur; do
    if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || { echo "enc $v failed"; exit 1; }
  done
done
unset WMX_LIB
timeout -k 10 200 python tools/enc_ab.py float8 >> $O/enc_ab.txt 2>&1 || { echo "enc8 failed"; exit 1; }
grep -v amdgpu.ids $O/enc_ab.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py bfloat16 \
  > $O/encprof.log 2>&1 || { echo encprof failed; exit 1; }
KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/enc_layer_breakdown.py "$KT" | tee $O/enc_layers.txt
