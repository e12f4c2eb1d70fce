#!/bin/bash
# round 4, GPU call 8: the mixed step at 16 windows (bf16) after the scratch fix, interleaved with the fast step
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04n}
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
  python -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];e=r['layer_e2e_us'];print('$tag', d['value'], d['stage_ms'][5], round(sum(e.values()),1), e)"
}
for i in 1 2 3; do
  run b16_base$i WMX_DEC_MIXED=0 -- --batch 16
  run b16_mixed$i WMX_DEC_MIXED=1 -- --batch 16
done
run b12_base WMX_DEC_MIXED=0 -- --batch 12
run b12_mixed WMX_DEC_MIXED=1 -- --batch 12
exit 0
