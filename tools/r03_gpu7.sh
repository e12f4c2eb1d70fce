#!/bin/bash
# round 3, GPU call 7: encoder attention with 8-wave (256-query) workgroups (half the K/V fill per query):
# encoder parity tests (default form), then an interleaved A/B of the three forms and the previous build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03h
mkdir -p $O
export PYTHONUNBUFFERED=1
L=$PWD/realtime-whisper-asr_amd/wmx
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_mx8.py tests/test_gpu_wide.py "tests/test_gpu_step.py::test_full_depth_large_v3_one_window" \
  > $O/enc_tests.log 2>&1
rc=$?; tail -3 $O/enc_tests.log
if [ $rc -ne 0 ]; then echo "encoder tests failed (rc $rc): stopping"; exit 1; fi
for r in 1 2; do
  WMX_LIB=$L/libwmx_base.so timeout -k 10 120 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || exit 1
  for f in 8 82 4; do
    WMX_ENC_ATTN=$f timeout -k 10 120 python tools/enc_ab.py bfloat16 2>&1 | sed "s/^/form $f /" >> $O/enc_ab.txt || exit 1
  done
done
grep -v amdgpu.ids $O/enc_ab.txt
