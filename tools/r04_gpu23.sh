#!/bin/bash
# round 4, GPU call 23: decode knobs re-measured with the groups in step (round 3 found them within the slow mode's
# noise): cross-attention key chunk, packed column tiles, separate cross-q, the mixed step
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04za}
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
  python -c "import json;d=json.load(open('$O/$tag.json'));m=d['decode_mode'];e=d['roofline']['layer_e2e_us'];print('$tag', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], round(sum(e.values()),1))"
}
if [ "${2:-}" = fold ]; then
  for i in 1 2; do
    run base_$i WMX_X=1 --
    run fold_$i WMX_FOLD=1 --
    run mlpf_$i WMX_MLP_FUSED=1 --
  done
  exit 0
fi
for i in 1 2; do
  run base_$i WMX_X=1 --
  run chunk768_$i WMX_CROSS_CHUNK=768 --
  run chunk512_$i WMX_CROSS_CHUNK=512 --
  run nctdd1_$i WMX_PACKED_NCT=1280:1280:1 --
  run nctqkv4_$i WMX_PACKED_NCT=3840:1280:4 --
  run xq0_$i WMX_XQ_FUSED=0 --
  run mixed_$i WMX_DEC_MIXED=1 --
done
exit 0
