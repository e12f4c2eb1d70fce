#!/bin/bash
# round 4, GPU call 4: fp8 cross-attention key chunk at 8 and 16 windows, and the packed GEMM's k-steps per wave
# (WMX_PACKED_PER) on the bf16 default line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04h}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
run() {  # tag, env-assignments..., then bench args after --
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream "$@" \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag', d['value'], d['stage_ms'][5], r['layer_e2e_us'])"
}
run f8b8_c512 WMX_CROSS_CHUNK=512 -- --dtype fp8 --batch 8
run f8b8_c768 WMX_CROSS_CHUNK=768 -- --dtype fp8 --batch 8
run f8b8_c1024 WMX_CROSS_CHUNK=1024 -- --dtype fp8 --batch 8
run f8b8_c1504 WMX_CROSS_CHUNK=1504 -- --dtype fp8 --batch 8
run f8b16_c512 WMX_CROSS_CHUNK=512 -- --dtype fp8 --task translate --batch 16
run f8b16_c1504 WMX_CROSS_CHUNK=1504 -- --dtype fp8 --task translate --batch 16
run bf8_per4 WMX_PACKED_PER=4 -- --batch 8
run bf8_per2 WMX_PACKED_PER=2 -- --batch 8
run bf8_per3 WMX_PACKED_PER=3 -- --batch 8
run bf8_per4b WMX_PACKED_PER=4 -- --batch 8
run bf8_per2b WMX_PACKED_PER=2 -- --batch 8
exit 0
