#!/bin/bash
# round 5, GPU call 4: the rank-local streaming path test; what the cross K / V and weight HBM streams cost with the
# groups in step (WMX_ABLATE 32 / 64 / 96: every layer reads layer 0's, timing only); a full default line with the
# sharded stream_load
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05d}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_e2e.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep "rank-local" $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2; do
  for ab in 0 32 64 96; do
    WMX_ABLATE=$ab timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_ab$ab.json 2> $O/b${i}_ab$ab.err || { echo "bench failed"; tail -5 $O/b${i}_ab$ab.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_ab$ab.json'));r=d['roofline'];print('b${i}_ab$ab', d['value'], d['ms_per_step'], d['stage_ms'][5], r['layer_e2e_us'])"
  done
done
timeout -k 10 600 python bench.py > $O/b_full.json 2> $O/b_full.err || { echo "bench failed"; tail -5 $O/b_full.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_full.json'));print('full', d['value'], d['roofline']['frac'], d.get('stream_load'), d.get('cpu_baseline'))"
exit 0
