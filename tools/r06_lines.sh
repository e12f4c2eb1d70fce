#!/bin/bash
# Round-6 secondary bench lines (run on the GPU box from the repo root): bash tools/r06_lines.sh <tag>
#   config 5 (fp8, translate, 16 windows per GPU) and the same shape in bf16; the int8 line (CTranslate2's grid)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:?tag}
mkdir -p "$O"
(while sleep 50; do date >> "$O/heartbeat.txt"; done) &
HB=$!
trap "kill $HB" EXIT
for spec in "fp8_b16:--dtype fp8 --task translate --batch 16" "bf16_b16:--task translate --batch 16" "int8:--dtype int8"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-stream $a > "$O/bench_$n.json" 2> "$O/bench_$n.err" || { echo "$n failed"; exit 1; }
  python - "$O/bench_$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["encoder"]["isolated_gpu_batch"]
print(sys.argv[2], d["value"], "decode_ms", d["stage_ms"][5], "enc_ms", e["ms"], "util", e["mfma_util"],
      "util_vs_dtype_peak", e.get("mfma_util_vs_dtype_peak"), "frac", d["roofline"]["frac"],
      "int8_rule" in d["config"])
PY
done
