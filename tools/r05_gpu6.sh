#!/bin/bash
# round 5, GPU call 6: the CTranslate2 int8 grid (model dtype I8) tests, then the fp8 and step / e2e suites on the
# rebuilt library (the packed GEMM's 8-bit template is now int8 or e4m3), and a default bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05f}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 500 --timeout-method thread -m gpu tests/test_gpu_int8.py > $O/tests_int8.log 2>&1
rc=$?; tail -2 $O/tests_int8.log; grep -E "int8 decode|int8 weights|worst" $O/tests_int8.log | head
if [ $rc -ne 0 ]; then echo "int8 tests failed"; grep -E "FAILED|Error|assert" $O/tests_int8.log | head -20; exit 1; fi
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mx8.py tests/test_gpu_e2e.py tests/test_gpu_checkpoint.py tests/test_gpu_concurrent.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b_def.json 2> $O/b_def.err || { echo "bench failed"; tail -5 $O/b_def.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_def.json'));print('default', d['value'], d['ms_per_step'], d['stage_ms'][5], d['roofline']['frac'])"
exit 0
