#!/bin/bash
# round 3 (session 2), GPU call 24: the 256 x 256 MX-fp8 GEMM (v_mfma_scale_f32_32x32x64_f8f6f4): lane-map probe,
# MX-fp8 parity tests, microbenchmark with and without it, encoder pass A/B (WMX_MX8_256=0 vs default)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zh}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 5 60 tools/mx8_check32 > $O/mx8_check32.txt 2>&1; cat $O/mx8_check32.txt
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py \
  > $O/tests.log 2>&1
rc=$?; grep -E "rel_l2|passed|failed|Error" $O/tests.log | tail -12
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
for v in 1 0; do
  echo "== WMX_MX8_256=$v" >> $O/mb.txt
  WMX_MX8_256=$v timeout -k 10 120 tools/mb_gemm256_cur >> $O/mb.txt 2>&1 || { echo "mb failed"; exit 1; }
done
grep -E "==|mx8" $O/mb.txt | sed -e 's/128x128.*| mx8/mx8/'
for r in 1 2 3; do
  for v in 0 1; do
    echo -n "WMX_MX8_256=$v " >> $O/enc_ab.txt
    WMX_MX8_256=$v timeout -k 10 200 python tools/enc_ab.py float8 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt || { echo "enc failed"; exit 1; }
  done
done
timeout -k 10 200 python tools/enc_ab.py bfloat16 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt
cat $O/enc_ab.txt
