#!/bin/bash
# round 3 (session 2), GPU call 31: decode mode, default vs WMX_FULL_CUMASK=1 (each context stream on a hardware queue of
# its own via an all-CU mask), 6 interleaved pairs of short bench runs
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zj}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
    || { echo "bench $n failed"; tail -5 $O/b.err; exit 1; }
  python - "$n" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:8s} {j['value']:8.2f}x decode {j['stage_ms'][5]:7.2f} ms mode {j['decode_mode']['mode']:5s} "
      f"ratio {j['decode_mode']['cross_to_chain_ratio']:.3f}")
PY
}
for r in 1 2 3 4 5 6; do
  run default WMX_X=1
  run fullmask WMX_FULL_CUMASK=1
done
