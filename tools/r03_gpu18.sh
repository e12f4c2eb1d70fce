#!/bin/bash
# round 3 (session 2), GPU call 18: per-layer kernel breakdown of the encoder pass, default library vs the one-phase
# gemm256 variant (libwmx_p1.so), twice each, interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03za}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2; do
  for v in base p1; do
    if [ $v = base ]; then unset WMX_LIB; else export WMX_LIB=$L/libwmx_$v.so; fi
    rm -rf /tmp/encprof
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py bfloat16 \
      > $O/encprof_$v.log 2>&1 || { echo encprof failed; exit 1; }
    KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
    echo "== $v $(grep encoder $O/encprof_$v.log)" | tee -a $O/layers.txt
    python3 tools/enc_layer_breakdown.py "$KT" | tee -a $O/layers.txt
  done
done
