#!/bin/bash
# round 3 (session 2), GPU call 34: encoder attention with a static priority for waves 4..7 (libwmx_aprio.so) vs the
# default: encoder parity on the variant, then the encoder pass (and the attention launch) interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zu}
mkdir -p $O
export PYTHONUNBUFFERED=1
L=$PWD/realtime-whisper-asr_amd/wmx
WMX_LIB=$L/libwmx_aprio.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py -k "wide_encoder" > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3 4; do
  for v in cur aprio; do
    if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py bfloat16 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt || { echo "enc $v failed"; exit 1; }
  done
done
cat $O/enc_ab.txt
