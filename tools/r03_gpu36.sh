#!/bin/bash
# round 3 (session 2), GPU call 36: LayerNorm -> MX-fp8 with two rows per wave (the default build)
# vs one row per wave (libwmx_lnr1.so): MX-fp8 parity on the default, the MX-fp8 encoder pass
# interleaved, and a kernel-trace summary of each
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zx}
mkdir -p $O
export PYTHONUNBUFFERED=1
L=$PWD/realtime-whisper-asr_amd/wmx
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3 4; do
  for v in cur lnr1; do
    if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py float8 2>&1 | grep -v amdgpu.ids >> $O/enc_ab.txt || { echo "enc $v failed"; exit 1; }
  done
done
cat $O/enc_ab.txt
export TMPDIR=/tmp
for v in cur lnr1; do
  if [ $v = cur ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 tools/enc_ab.py \
    float8 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
done
find $O -name '*kernel_trace.csv' -delete
grep -h layernorm_mx8 $O/prof_*/*/*kernel_stats.csv $O/prof_*/*kernel_stats.csv 2>/dev/null
exit 0
