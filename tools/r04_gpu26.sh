#!/bin/bash
# round 4, GPU call 26: config-5 line knobs with the groups in step: split target and fp8 cross-attention chunk
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04ze}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
run() {
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream --dtype fp8 --task translate --batch 16 "$@" \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));m=d['decode_mode'];e=d['roofline']['layer_e2e_us'];print('$tag', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], round(sum(e.values()),1))"
}
for i in 1 2; do
  run base_$i WMX_X=1 --
  run t320_$i WMX_PACKED_TARGET=320 --
  run t640_$i WMX_PACKED_TARGET=640 --
  run c768_$i WMX_CROSS_CHUNK=768 --
  run c1024_$i WMX_CROSS_CHUNK=1024 --
done
exit 0
