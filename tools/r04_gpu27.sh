#!/bin/bash
# round 4, GPU call 27: the single-stream latency line (one context, beam 5, R = 5 rows: every launch boundary
# exposed) under the step variants with fewer launches: default vs mixed vs folded
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zh}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for v in base mixed fold base; do
  E=WMX_X=1; [ $v = mixed ] && E=WMX_DEC_MIXED=1; [ $v = fold ] && E=WMX_FOLD=1
  env $E timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { echo "$v failed"; tail -3 $O/$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$v.json'));print('$v', d['value'], [(s['model'], s['p50_ms'], s['decode_steps_per_call']) for s in d['stream_latency']], d['stream_load']['p50_ms'])"
done
exit 0
