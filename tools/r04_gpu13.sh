#!/bin/bash
# round 4, GPU call 13: split-K partial store policy (plain / non-temporal / write-through sc1), interleaved default
# bench lines; the variant libraries are selected with WMX_LIB
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04s}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
L=$PWD/realtime-whisper-asr_amd/wmx
run() {
  local tag=$1 lib=$2
  WMX_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];e=r['layer_e2e_us'];print('$tag', d['value'], d['stage_ms'][5], round(sum(e.values()),1), {k: e[k] for k in e if 'reduce' in k or k in ('dec_out','dec_fc2','dec_qkv')})"
}
for i in 1 2 3; do
  run p0_$i libwmx.so
  run p1_$i libwmx_pst1.so
  run p2_$i libwmx_pst2.so
done
exit 0
