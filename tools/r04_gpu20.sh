#!/bin/bash
# round 4, GPU call 20: does a small enforced phase offset between the in-step groups (group 1 starts X us after
# group 0, after the lockstep barrier) persist, and is it faster than lockstep (cross attentions interleaved with the
# other group's weight-streaming launches instead of coinciding)?
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04z5}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for x in 0 10 20 40 80 0; do
  timeout -k 10 240 python tools/phase_probe.py --calls 3 --lockstep 1 --phase-offset-us $x --out $O/ph_x$x.json > $O/ph_x$x.log 2>&1 \
    || { echo "probe $x failed"; tail -5 $O/ph_x$x.log; exit 1; }
  python -c "
import json;r=json.load(open('$O/ph_x$x.json'));print('x$x', [(x['decode_ms'], x['offset_us_median'], x['offset_us_min_max']) for x in r])"
done
exit 0
