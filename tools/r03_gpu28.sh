#!/bin/bash
# round 3 (session 2), GPU call 28: GELU -> MX-fp8 epilogue with one MX block per thread in the 256 x 256 MX-fp8 GEMM:
# MX-fp8 parity, then the MX-fp8 encoder pass interleaved against libwmx_prev.so and a per-layer breakdown
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zn}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py > $O/tests.log 2>&1
rc=$?; grep -E "rel_l2|passed|failed|Error" $O/tests.log | tail -8
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3; do
  for v in prev cur; do
    if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py float8 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt || { echo "enc $v failed"; exit 1; }
  done
done
unset WMX_LIB
cat $O/enc_ab.txt
rm -rf /tmp/encprof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py float8 \
  > $O/encprof.log 2>&1 || { echo encprof failed; exit 1; }
KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/enc_layer_breakdown.py "$KT" | tee $O/enc_layers.txt
