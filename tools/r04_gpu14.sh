#!/bin/bash
# round 4, GPU call 14: the two context groups' relative phase per call (tools/phase_probe.py), five fresh processes
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04t}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3 4 5; do
  echo "process $i"
  timeout -k 10 240 python tools/phase_probe.py --calls 4 --out $O/run$i.json > $O/run$i.log 2>&1 || { echo "run $i failed"; tail -5 $O/run$i.log; exit 1; }
  grep '^{' $O/run$i.log
done
exit 0
