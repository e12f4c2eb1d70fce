#!/bin/bash
# round 4, GPU call 17: lockstep A/B on the phase probe: decode-start barrier (1), none (0), every chunk (2); the
# offset between the groups per chunk shows whether and when they unlock
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04x}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3 4; do
  for ls in 0 1; do
    ch=0; l=$ls; if [ $ls = 2 ]; then ch=1; l=1; fi
    WMX_LOCKSTEP_CHUNKS=$ch timeout -k 10 240 python tools/phase_probe.py --calls 4 --lockstep $l --out $O/ph${i}_ls$ls.json > $O/ph${i}_ls$ls.log 2>&1 \
      || { echo "probe $i $ls failed"; tail -5 $O/ph${i}_ls$ls.log; exit 1; }
    python -c "
import json;r=json.load(open('$O/ph${i}_ls$ls.json'));print('ph${i}_ls$ls', [(x['decode_ms'][0], x['offset_us_median'], x['offset_us_min_max']) for x in r])"
  done
done
exit 0
