#!/bin/bash
# round 3 (session 2), GPU call 22: decode cross attention spread over more CUs: the separate cross-q launch with 512- /
# 384-key chunks (320 / 400 workgroups per group) vs the fused default, interleaved bench runs
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zf}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
    || { echo "bench $n failed"; tail -5 $O/b.err; exit 1; }
  python - "$n" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
l = j["roofline"]["layer_e2e_us"]
print(f"{sys.argv[1]:10s} {j['value']:8.2f}x decode {j['stage_ms'][5]:7.2f} ms mode {j['decode_mode']['mode']:5s} "
      f"cross {l['cross_attn']:6.2f} us chain {sum(l.values()):6.2f} us")
PY
}
for r in 1 2; do
  run default WMX_X=1
  run unf512 WMX_XQ_FUSED=0 WMX_CROSS_CHUNK=512
  run unf384 WMX_XQ_FUSED=0 WMX_CROSS_CHUNK=384
  run fus512 WMX_CROSS_CHUNK=512
done
