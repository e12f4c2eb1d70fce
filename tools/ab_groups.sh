#!/bin/bash
# Context-group / hardware-queue A/B: bash tools/ab_groups.sh <outdir> "<name> <ENV=V ...|-> -- <bench args>" ...
set -e
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%% *}; rest=${spec#* }
  envs=${rest%% -- *}; args=${rest#* -- }
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-stream --steps 4 $args > "$out/$name.log" 2>&1
  python -c "
import json
l=[x for x in open('$out/$name.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$name', d['value'], d['ms_per_step'], d['stage_ms'][5])"
done
