#!/bin/bash
# round 3 (session 2), GPU call 17: gemm256 main loop with one 32-MFMA segment per slice (WMX_G256_PHASES=1) vs the
# two-phase form: microbenchmark (correctness vs the 128 tile, TF/s, per-tile stamps) interleaved, then the encoder
# pass of the library variant vs the default library interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03z}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in p2 p1; do
    echo "== $v" >> $O/mb.txt
    timeout -k 10 120 tools/mb_gemm256_$v >> $O/mb.txt 2>&1 || { echo "mb $v failed"; cat $O/mb.txt; exit 1; }
  done
done
for v in p2s p1s; do
  echo "== $v" >> $O/mb.txt
  timeout -k 10 120 tools/mb_gemm256_$v >> $O/mb.txt 2>&1 || { echo "mb $v failed"; exit 1; }
done
grep -E "==|256x256|stamps|PASS|FAIL" $O/mb.txt | sed -e 's/128x128.*| 256x256/256:/' -e 's/maxdiff.*//'
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3; do
  for v in base p1; do
    if [ $v = base ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    timeout -k 10 200 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || { echo "enc $v failed"; exit 1; }
  done
done
grep -v amdgpu.ids $O/enc_ab.txt
