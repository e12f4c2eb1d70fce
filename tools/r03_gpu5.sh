#!/bin/bash
# round 3, GPU call 5: the fused decode MLP (WMX_MLP_FUSED=1): one short guarded parity run first, then the full
# parity rerun, then an interleaved bench A/B against the split form
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03e
mkdir -p $O
export PYTHONUNBUFFERED=1
WMX_MLP_FUSED=1 timeout -k 10 150 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_step.py -k "forced_steps_wide_beam5" > $O/first.log 2>&1
rc=$?; tail -3 $O/first.log
if [ $rc -ne 0 ]; then echo "fused MLP first run failed (rc $rc): stopping"; exit 1; fi
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 890 --timeout-method thread -m gpu tests/test_gpu_step.py \
  -k fused_mlp > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log
if [ $rc -ne 0 ]; then echo "fused MLP parity failed (rc $rc): stopping"; exit 1; fi
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stream > $O/split_$r.json 2> $O/split_$r.err \
    || { echo split bench failed; exit 1; }
  WMX_MLP_FUSED=1 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stream > $O/fused_$r.json \
    2> $O/fused_$r.err || { echo fused bench failed; exit 1; }
  python - $O/split_$r.json $O/fused_$r.json <<'PY'
import json, sys
for p in sys.argv[1:]:
    j = json.loads(open(p).read().strip().splitlines()[-1])
    print(p.split("/")[-1], j["value"], j["ms_per_step"], "decode stage ms", j["stage_ms"][5], j.get("decode_mode"))
PY
done
exit 0
