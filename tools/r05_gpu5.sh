#!/bin/bash
# round 5, GPU call 5: the cross attention with every wave's query-projection loads issued before any K load
# (WMX_XATTN_ISSUE_BAR=1): parity (step tests), interleaved bench lines, and its phase stamps
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05e}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
WMX_XATTN_ISSUE_BAR=1 timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_step.py -k "wide or large_v3 or concurrent" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2 3; do
  for ib in 1 0; do
    WMX_XATTN_ISSUE_BAR=$ib timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_ib$ib.json 2> $O/b${i}_ib$ib.err || { echo "bench failed"; tail -5 $O/b${i}_ib$ib.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_ib$ib.json'));r=d['roofline'];print('b${i}_ib$ib', d['value'], d['ms_per_step'], d['stage_ms'][5], r['layer_e2e_us']['cross_attn'])"
  done
done
WMX_XATTN_ISSUE_BAR=1 WMX_PHASE_PROBE=1 WMX_PHASE_DUMP=$O/phases.npz timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline --no-stream > $O/b_phase.json 2> $O/b_phase.err || { echo "bench failed"; tail -5 $O/b_phase.err; exit 1; }
python tools/xattn_phases.py $O/phases.npz
exit 0
