#!/bin/bash
# round 4, GPU call 21: split-K workgroup target (WMX_PACKED_TARGET 480 default vs 240 / 320: fewer slices = less
# partial traffic) under the lockstep start, interleaved default bench lines
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04z6}
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
  python -c "import json;d=json.load(open('$O/$tag.json'));m=d['decode_mode'];e=d['roofline']['layer_e2e_us'];print('$tag', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], round(sum(e.values()),1), {k: e[k] for k in e if k.startswith('dec_') or k.startswith('reduce')})"
}
if [ "${2:-}" = sweep2 ]; then
  for i in 1 2; do
    run t240_$i WMX_PACKED_TARGET=240 --
    run t200_$i WMX_PACKED_TARGET=200 --
    run t160_$i WMX_PACKED_TARGET=160 --
    run t120_$i WMX_PACKED_TARGET=120 --
  done
  run f8_t480 WMX_PACKED_TARGET=480 -- --dtype fp8 --task translate --batch 16
  run f8_t240 WMX_PACKED_TARGET=240 -- --dtype fp8 --task translate --batch 16
  run f8_t160 WMX_PACKED_TARGET=160 -- --dtype fp8 --task translate --batch 16
  run b16_t480 WMX_PACKED_TARGET=480 -- --batch 16
  run b16_t240 WMX_PACKED_TARGET=240 -- --batch 16
  exit 0
fi
for i in 1 2 3; do
  run t480_$i WMX_PACKED_TARGET=480 --
  run t240_$i WMX_PACKED_TARGET=240 --
  run t320_$i WMX_PACKED_TARGET=320 --
done
exit 0
