#!/bin/bash
# round 4, GPU call 3: the full default bench line (stream latency + the new under-load stream entry + CPU baseline),
# then the fp8 16-window line with other cross-attention key chunks (WMX_CROSS_CHUNK)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04g}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail -5 $O/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['stage_ms']);print(json.dumps(d.get('stream_latency')));print(json.dumps(d.get('stream_load')));print(d.get('cpu_baseline'))"
run() {  # tag, env..., -- args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream --dtype fp8 --task translate --batch 16 \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag', d['value'], d['stage_ms'], r['layer_e2e_us'].get('cross_attn'))"
}
run fp8_c1024 WMX_CROSS_CHUNK=1024
run fp8_c512 WMX_CROSS_CHUNK=512
run fp8_c768 WMX_CROSS_CHUNK=768
run fp8_c1504 WMX_CROSS_CHUNK=1504
run fp8_c1024b WMX_CROSS_CHUNK=1024
exit 0
