#!/bin/bash
# round 5, GPU call 2: the new decode-loop NaN-guard tests and the relative fp8 alignment bounds; the cross
# attention's phase stamps in the default bench workload (diagnostics), against a default line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05b}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu "tests/test_gpu_mx8.py::test_fp8_decode_word_alignment_large_v3_heads" tests/test_gpu_align.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "decode step|window [01]|fp8 / bf16|excess" $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; fi
WMX_PHASE_PROBE=1 WMX_PHASE_DUMP=$O/phases.npz timeout -k 10 300 python bench.py --steps 2 --no-cpu-baseline --no-stream > $O/b_phase.json 2> $O/b_phase.err || { echo "bench failed"; tail -5 $O/b_phase.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_phase.json'));print('phase', d['value'], d['ms_per_step'], d['stage_ms'], d['roofline']['layer_e2e_us']['cross_attn'])"
python tools/xattn_phases.py $O/phases.npz
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b_def.json 2> $O/b_def.err || { echo "bench failed"; tail -5 $O/b_def.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_def.json'));print('default', d['value'], d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d['roofline']['frac_span'])"
exit 0
