#!/bin/bash
# round 3 (session 2), GPU call 29: block-per-thread folded-LN residual epilogue (gemm256 RESID32_LNS): encoder
# parity, then the encoder pass interleaved against libwmx_prev.so (HEAD without it) and a per-layer breakdown
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zm}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wide.py \
  tests/test_gpu_step.py tests/test_gpu_parity.py -k "wide_encoder or encoder_layernorm_fold or small_models or wide_decoder or encoder_matches" \
  > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" $O/tests.log | tail -3
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3; do
  for v in prev cur; do
    if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py bfloat16 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt || { echo "enc $v failed"; exit 1; }
  done
done
unset WMX_LIB
cat $O/enc_ab.txt
rm -rf /tmp/encprof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py bfloat16 \
  > $O/encprof.log 2>&1 || { echo encprof failed; exit 1; }
KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/enc_layer_breakdown.py "$KT" | tee $O/enc_layers.txt
