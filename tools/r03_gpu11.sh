#!/bin/bash
# round 3, GPU call 11: the word-alignment forward's GEMMs (M ~ 900 rows per group) on 128 x 128 tiles
# (WMX_GEMM_M128=512) against the default 64 x 64: interleaved bench A/B of the align stage and the whole call
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03r
mkdir -p $O
for r in 1 2 3; do
  for v in 1024 512; do
    WMX_GEMM_M128=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
      || { echo "bench $v failed"; exit 1; }
    python - "$v" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"M128={sys.argv[1]:5s} {j['value']:8.2f}x stages {j['stage_ms']} mode {j['decode_mode']['mode']}")
PY
  done
done
