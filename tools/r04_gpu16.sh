#!/bin/bash
# round 4, GPU call 16: lockstep decode start (host barrier before the decode loop) -- phase probe processes with and
# without it, then interleaved default bench lines (WMX_LOCKSTEP=1 default vs 0)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04w}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3 4; do
  for ls in 1 0; do
    timeout -k 10 240 python tools/phase_probe.py --calls 4 --lockstep $ls --out $O/ph${i}_ls$ls.json > $O/ph${i}_ls$ls.log 2>&1 \
      || { echo "probe $i $ls failed"; tail -5 $O/ph${i}_ls$ls.log; exit 1; }
    python -c "
import json;r=json.load(open('$O/ph${i}_ls$ls.json'));print('ph${i}_ls$ls', [(x['decode_ms'][0], x['offset_us_median']) for x in r])"
  done
done
for i in 1 2 3; do
  for ls in 1 0; do
    WMX_LOCKSTEP=$ls timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_ls$ls.json 2> $O/b${i}_ls$ls.err || { echo "bench failed"; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_ls$ls.json'));m=d['decode_mode'];print('b${i}_ls$ls', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']])"
  done
done
exit 0
