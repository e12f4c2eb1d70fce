#!/bin/bash
# round 4, GPU call 19: context-group count again, now with the lockstep start (groups share weight reads when in
# step): 8 windows as 2 groups (4 HW queues) vs 4 groups (8 HW queues), interleaved; then 16 windows
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04z4}
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
  python -c "import json;d=json.load(open('$O/$tag.json'));m=d['decode_mode'];print('$tag', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']])"
}
for i in 1 2; do
  run b8_g2_$i GPU_MAX_HW_QUEUES=4 -- --groups 2
  run b8_g4q8_$i GPU_MAX_HW_QUEUES=8 -- --groups 4
done
run b16_g2 GPU_MAX_HW_QUEUES=4 -- --batch 16 --groups 2
run b16_g4q8 GPU_MAX_HW_QUEUES=8 -- --batch 16 --groups 4
run f8b16_g2 GPU_MAX_HW_QUEUES=4 -- --dtype fp8 --task translate --batch 16 --groups 2
run f8b16_g4q8 GPU_MAX_HW_QUEUES=8 -- --dtype fp8 --task translate --batch 16 --groups 4
exit 0
