#!/bin/bash
# round 5, GPU call 3: the window-pair cross attention (WPW = 2): decode parity tests, then interleaved bench lines
# pairs on / off, and the phase stamps of the new form
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05c}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_concurrent.py tests/test_gpu_e2e.py tests/test_gpu_align.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
for i in 1 2; do
  for pr in 1 0; do
    WMX_XATTN_PAIRS=$pr timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_p$pr.json 2> $O/b${i}_p$pr.err || { echo "bench failed"; tail -5 $O/b${i}_p$pr.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_p$pr.json'));r=d['roofline'];print('b${i}_p$pr', d['value'], d['ms_per_step'], d['stage_ms'][5], r['frac'], r['layer_e2e_us'])"
  done
done
WMX_PHASE_PROBE=1 WMX_PHASE_DUMP=$O/phases.npz timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline --no-stream > $O/b_phase.json 2> $O/b_phase.err || { echo "bench failed"; tail -5 $O/b_phase.err; exit 1; }
python tools/xattn_phases.py $O/phases.npz
exit 0
