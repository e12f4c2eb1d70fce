#!/bin/bash
# round 4, GPU call 15: phase probe processes interleaved with default bench lines (catch a slow-mode run)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04u}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3; do
  timeout -k 10 240 python tools/phase_probe.py --calls 3 --out $O/ph$i.json > $O/ph$i.log 2>&1 || { echo "probe $i failed"; tail -5 $O/ph$i.log; exit 1; }
  python -c "
import json;r=json.load(open('$O/ph$i.json'));print('ph$i', [(x['decode_ms'], x['phase_median'], x['offset_us_median']) for x in r])"
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b$i.json 2> $O/b$i.err || { echo "bench $i failed"; exit 1; }
  python -c "import json;d=json.load(open('$O/b$i.json'));m=d['decode_mode'];print('b$i', d['value'], m['groups'], m['cross_to_chain_ratio'])"
done
exit 0
