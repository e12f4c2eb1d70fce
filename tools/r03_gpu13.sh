#!/bin/bash
# round 3, GPU call 13: each context group on its own half of the CUs (WMX_CU_SPLIT=2: CU mask i mod 2 == group)
# against the shared default: interleaved bench A/B (decode time and mode)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03u
mkdir -p $O
for r in 1 2 3; do
  for v in 0 2; do
    WMX_CU_SPLIT=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
      || { echo "bench $v failed"; tail -5 $O/b.err; exit 1; }
    python - "$v" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = j["roofline"]["layer_e2e_us"]
print(f"split={sys.argv[1]} {j['value']:8.2f}x {j['ms_per_step']:7.2f} ms stages {j['stage_ms']} mode {j['decode_mode']['mode']} "
      f"ratio {j['decode_mode']['cross_to_chain_ratio']} cross {e.get('cross_attn')} fc1 {e.get('dec_fc1')}")
PY
  done
done
