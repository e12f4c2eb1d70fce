#!/bin/bash
# round 4, GPU call 1: the fp8 decode (8-bit decoder weights + fp8 cross-K/V images) -- parity tests first, then the
# non-finite guard, the parameter-region broadcast, and the 16-window bench lines fp8 vs bf16
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04a}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py \
  tests/test_gpu_e2e.py tests/test_gpu_rccl.py tests/test_gpu_concurrent.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed (rc $rc)"; grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; fi
timeout -k 10 300 python bench.py --dtype fp8 --task translate --batch 16 --steps 3 --no-cpu-baseline --no-stream \
  > $O/bench_fp8_b16.json 2> $O/bench_fp8_b16.err || { echo fp8 bench failed; tail -5 $O/bench_fp8_b16.err; exit 1; }
head -c 400 $O/bench_fp8_b16.json; echo
timeout -k 10 300 python bench.py --batch 16 --steps 3 --no-cpu-baseline --no-stream > $O/bench_bf16_b16.json \
  2> $O/bench_bf16_b16.err || { echo bf16 b16 bench failed; exit 1; }
head -c 400 $O/bench_bf16_b16.json; echo
exit 0
