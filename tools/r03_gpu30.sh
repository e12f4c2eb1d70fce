#!/bin/bash
# round 3 (session 2), GPU call 30: does the decode's slow mode follow the chip state?  Short bench runs fresh, right
# after 150 s of back-to-back encoder passes, and after a 60 s idle pause (GPU temperature read with rocm-smi)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zq}
mkdir -p $O
export PYTHONUNBUFFERED=1
temp() { timeout 30 rocm-smi --showtemp 2>/dev/null | grep -iE "junction|edge|memory" | head -3 | tr -s ' ' | tee -a $O/ab.txt; }
run() {
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
    || { echo "bench failed"; tail -5 $O/b.err; exit 1; }
  python - "$1" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:10s} {j['value']:8.2f}x decode {j['stage_ms'][5]:7.2f} ms mode {j['decode_mode']['mode']:5s} "
      f"ratio {j['decode_mode']['cross_to_chain_ratio']:.3f} enc8 {j['encoder']['isolated_gpu_batch']['ms']:.2f} ms")
PY
}
temp; run fresh; run fresh
timeout -k 10 300 python tools/heat_load.py 150 > $O/heat.log 2>&1 || { echo heat failed; exit 1; }
tail -1 $O/heat.log | tee -a $O/ab.txt
temp; run hot; run hot2
sleep 60
temp; run rested; run rested2
