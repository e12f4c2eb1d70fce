#!/bin/bash
# round 3, GPU call 14: the beam step tail in one launch (beam_tail_kernel): the step / search / concurrency /
# end-to-end GPU tests first, then an interleaved bench A/B against libwmx_base.so (the separate kernels)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03v
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_step.py \
  tests/test_gpu_concurrent.py tests/test_gpu_align.py tests/test_gpu_e2e.py -k "not fused_mlp" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc): stopping"; exit 1; fi
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3 4; do
  for v in base new; do
    if [ $v = base ]; then export WMX_LIB=$L/libwmx_base.so; else unset WMX_LIB; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
      || { echo "bench $v failed"; exit 1; }
    python - "$v" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:5s} {j['value']:8.2f}x {j['ms_per_step']:7.2f} ms decode {j['stage_ms'][5]:7.2f} mode {j['decode_mode']['mode']}")
PY
  done
done
