#!/bin/bash
# round 3 (session 2), GPU call 16: encoder LayerNorm fold -- smoke, the encoder parity tests that reach the fold (large-v3
# width 3 windows, full-depth large-v3 3 windows vs the unfolded model, base / tiny full depth), then an interleaved
# encoder-pass A/B against libwmx_base.so (HEAD before the fold) and a per-layer kernel breakdown of the folded pass
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03x}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wide.py \
  tests/test_gpu_step.py -k "wide_encoder or encoder_layernorm_fold or small_models or wide_decoder" > $O/tests.log 2>&1
rc=$?; grep -E "rel_l2|passed|failed|Error" $O/tests.log | tail -20
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export WMX_LIB=$L/libwmx_base.so; else unset WMX_LIB; fi
    timeout -k 10 200 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || { echo "enc $v failed"; exit 1; }
  done
done
unset WMX_LIB
cat $O/enc_ab.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/encprof -o run -- python3 tools/encprof.py bfloat16 \
  > $O/encprof.log 2>&1 || { echo encprof failed; exit 1; }
KT=$(find /tmp/encprof -name "run_kernel_trace.csv" -print -quit)
python3 tools/enc_layer_breakdown.py "$KT" | tee $O/enc_layers.txt
