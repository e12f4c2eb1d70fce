#!/bin/bash
# round 3, GPU call 2: the re-worked beam-options tests (and the folded-step rerun that includes them), the new
# parity tests with their printed metrics, an f16 bench line and a default bench line with the decode mode
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_step.py -k "beam_options or folded" \
  > $O/step_options.log 2>&1
rc=$?; tail -5 $O/step_options.log
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_align.py tests/test_gpu_concurrent.py \
  "tests/test_gpu_parity.py::test_word_alignment_matrix_micro" "tests/test_gpu_parity.py::test_greedy_transcribe_matches_oracle" \
  tests/test_gpu_mx8.py tests/test_gpu_rccl.py > $O/new_tests.log 2>&1
rc2=$?; tail -3 $O/new_tests.log
timeout -k 10 300 python bench.py --dtype f16 --steps 5 --no-cpu-baseline --no-stream > $O/bench_f16.json 2> $O/bench_f16.err
echo "f16 bench rc $?"; head -c 400 $O/bench_f16.json; echo
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream > $O/bench_bf16.json 2> $O/bench_bf16.err
echo "bf16 bench rc $?"; head -c 400 $O/bench_bf16.json; echo
exit $((rc + rc2))
