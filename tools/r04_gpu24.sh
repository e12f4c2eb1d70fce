#!/bin/bash
# round 4, GPU call 24: the packed GEMM's LDS budget with two groups in step (a 160 KiB reduction image allows one
# workgroup per CU; two groups' launches at once may exceed 256): WMX_PACKED_LDS80=1 vs default, 8 and 16 windows
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zb}
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
  python -c "import json;d=json.load(open('$O/$tag.json'));m=d['decode_mode'];e=d['roofline']['layer_e2e_us'];print('$tag', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], round(sum(e.values()),1), {k: e[k] for k in ('dec_fc1','dec_fc2','dec_qkv')})"
}
if [ "${2:-}" = b16 ]; then
  for i in 1 2; do
    run f8_base_$i WMX_X=1 -- --dtype fp8 --task translate --batch 16
    run f8_lds80_$i WMX_PACKED_LDS80=1 -- --dtype fp8 --task translate --batch 16
    run b16_base_$i WMX_X=1 -- --batch 16
    run b16_lds80_$i WMX_PACKED_LDS80=1 -- --batch 16
  done
  exit 0
fi
for i in 1 2; do
  run base_$i WMX_X=1 --
  run lds80_$i WMX_PACKED_LDS80=1 --
done
run f8_base WMX_X=1 -- --dtype fp8 --task translate --batch 16
run f8_lds80 WMX_PACKED_LDS80=1 -- --dtype fp8 --task translate --batch 16
exit 0
