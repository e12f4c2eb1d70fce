#!/bin/bash
# round 3 (session 2), GPU call 21: a 5-slot gemm256 ring (4 slices in flight) for the kinds without the folded-LN
# statistics (out-proj, fc2, conv, cross-K/V): encoder parity on the variant library, microbenchmark 4 vs 5 slots,
# encoder pass interleaved (default vs libwmx_s5.so) with a per-layer breakdown of each
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03ze}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/realtime-whisper-asr_amd/wmx
WMX_LIB=$L/libwmx_s5.so timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py tests/test_gpu_step.py -k "wide_encoder or encoder_layernorm_fold or wide_decoder or small_models" \
  > $O/tests_s5.log 2>&1
rc=$?; grep -E "passed|failed|Error" $O/tests_s5.log | tail -3
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
for v in s4 s5 s4 s5; do
  echo "== $v" >> $O/mb.txt
  timeout -k 10 120 tools/mb_gemm256_$v >> $O/mb.txt 2>&1 || { echo "mb $v failed"; exit 1; }
done
grep -E "==|256x256|PASS|FAIL" $O/mb.txt | sed -e 's/128x128.*| 256x256/256:/' -e 's/maxdiff.*//'
for r in 1 2 3; do
  for v in cur s5; do
    if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || { echo "enc $v failed"; exit 1; }
  done
done
grep -v amdgpu.ids $O/enc_ab.txt
for v in cur s5; do
  if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
  rm -rf /tmp/encprof
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py bfloat16 \
    > $O/encprof_$v.log 2>&1 || { echo encprof failed; exit 1; }
  KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
  echo "== $v" | tee -a $O/layers.txt
  python3 tools/enc_layer_breakdown.py "$KT" | tee -a $O/layers.txt
done
