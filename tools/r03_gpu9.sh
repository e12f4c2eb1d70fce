#!/bin/bash
# round 3, GPU call 9: the in-wave software-pipelined encoder attention (WMX_ENC_ATTN=15 / 158): encoder parity
# tests with it, then an interleaved A/B against the default 8-wave form
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03n
mkdir -p $O
export PYTHONUNBUFFERED=1
WMX_ENC_ATTN=15 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "encoder" > $O/t15_first.log 2>&1
rc=$?; tail -3 $O/t15_first.log
if [ $rc -ne 0 ]; then echo "t15 first test failed (rc $rc): stopping"; exit 1; fi
for f in 15 158; do
  WMX_ENC_ATTN=$f timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "not alignment_matrix and not fused_reduce_ln" \
    tests/test_gpu_mx8.py tests/test_gpu_wide.py "tests/test_gpu_step.py::test_full_depth_large_v3_one_window" \
    > $O/enc_tests_$f.log 2>&1
  rc=$?; tail -2 $O/enc_tests_$f.log
  if [ $rc -ne 0 ]; then echo "encoder tests with form $f failed (rc $rc): stopping"; exit 1; fi
done
for r in 1 2; do
  for f in 8 15 158; do
    WMX_ENC_ATTN=$f timeout -k 10 120 python tools/enc_ab.py bfloat16 2>&1 | grep -v amdgpu.ids | sed "s/^/form $f /" >> $O/enc_ab.txt || exit 1
  done
done
cat $O/enc_ab.txt
