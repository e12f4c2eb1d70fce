#!/bin/bash
# round 4, GPU call 11: context-group count with more hardware queues (16-window fp8 / bf16, 8-window bf16)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04q}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
run() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream "$@" \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['stage_ms'])"
}
run f8b16_g2 GPU_MAX_HW_QUEUES=4 -- --dtype fp8 --task translate --batch 16 --groups 2
run f8b16_g4q8 GPU_MAX_HW_QUEUES=8 -- --dtype fp8 --task translate --batch 16 --groups 4
run f8b16_g2q8 GPU_MAX_HW_QUEUES=8 -- --dtype fp8 --task translate --batch 16 --groups 2
run b8_g2 GPU_MAX_HW_QUEUES=4 -- --groups 2
run b8_g3q8 GPU_MAX_HW_QUEUES=8 -- --groups 3
run b8_g4q8 GPU_MAX_HW_QUEUES=8 -- --groups 4
exit 0
