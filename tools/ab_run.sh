#!/bin/bash
# Interleaved A/B of bench.py under environment variants on one box.
# usage: bash tools/ab_run.sh <outdir> "<name> <ENV=V ...>" ...   (use "-" for no environment)
set -e
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%% *}; envs=${spec#* }
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-stream --steps ${AB_STEPS:-5} > "$out/$name.log" 2>&1
  python - "$out/$name.log" "$name" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["ms_per_step"], d["stage_ms"][5], d["roofline"]["achieved"], flush=True)
PY
done
