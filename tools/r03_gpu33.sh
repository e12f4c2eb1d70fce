#!/bin/bash
# round 3 (session 2), GPU call 33: static priority for the lagging half in all three ping-pong GEMMs (default now)
# against the per-segment s_setprio build (libwmx_prio0.so): bf16 and MX-fp8 encoder passes interleaved; parity
# of the MX-fp8 and encoder tests on the default build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zt}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py \
  tests/test_gpu_wide.py -k "mx8 or wide_encoder" > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L=$PWD/realtime-whisper-asr_amd/wmx
for dt in bfloat16 float8; do
  for r in 1 2 3; do
    for v in prio0 cur; do
      if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
      timeout -k 10 200 python tools/enc_ab.py $dt 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt || { echo "enc $v failed"; exit 1; }
    done
  done
done
cat $O/enc_ab.txt
