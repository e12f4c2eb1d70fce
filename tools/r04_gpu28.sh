#!/bin/bash
# round 4, GPU call 28: encoder / remaining knobs with the groups in step: encoder attention form (8 default, 4, 82),
# cross-attention XCD remap, packed waves per k-step target
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zi}
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
  python -c "import json;d=json.load(open('$O/$tag.json'));m=d['decode_mode'];iso=d['encoder']['isolated_gpu_batch'];print('$tag', d['value'], d['ms_per_step'], d['stage_ms'][1], [g['decode_stage_ms'] for g in m['groups']], iso.get('ms'), iso.get('mfma_util'))"
}
for i in 1 2; do
  run base_$i WMX_X=1 --
  run ea4_$i WMX_ENC_ATTN=4 --
  run ea82_$i WMX_ENC_ATTN=82 --
  run remap_$i WMX_XATTN_REMAP=1 --
  run per2_$i WMX_PACKED_PER=2 --
done
exit 0
