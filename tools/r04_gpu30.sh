#!/bin/bash
# round 4, GPU call 30: the default bench line five times on one box (the spread of the headline with the groups in
# step), exactly as the driver runs it (python bench.py, no flags)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04zk}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3 4 5; do
  timeout -k 10 400 python bench.py > $O/b$i.json 2> $O/b$i.err || { echo "bench failed"; exit 1; }
  python -c "import json;d=json.load(open('$O/b$i.json'));m=d['decode_mode'];print('b$i', d['value'], d['ms_per_step'], [g['decode_stage_ms'] for g in m['groups']], d['roofline']['frac'], d['encoder']['isolated_gpu_batch']['mfma_util'])"
done
exit 0
