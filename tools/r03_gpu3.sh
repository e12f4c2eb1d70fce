#!/bin/bash
# round 3, GPU call 3: stream-K GEMM parity + encoder A/B (base = HEAD before stream-K, new with / without the
# split), the re-worked beam-options tests and the new parity tests with their printed metrics, bench lines
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03c
mkdir -p $O
export PYTHONUNBUFFERED=1
L=$PWD/realtime-whisper-asr_amd/wmx
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread tests/test_gpu_streamk.py > $O/streamk.log 2>&1
rc=$?; tail -4 $O/streamk.log
if [ $rc -ne 0 ]; then echo "stream-K test failed: stopping before the A/B"; exit 1; fi
for r in 1 2 3; do
  WMX_LIB=$L/libwmx_base.so timeout -k 10 120 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/enc_ab.py bfloat16 >> $O/enc_ab.txt 2>&1 || exit 1
  WMX_G256_SK=0 timeout -k 10 120 python tools/enc_ab.py bfloat16 | sed 's/^/SK0 /' >> $O/enc_ab.txt 2>&1 || exit 1
done
cat $O/enc_ab.txt
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_step.py -k "beam_options or folded" \
  > $O/step_options.log 2>&1
rc1=$?; tail -3 $O/step_options.log
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_align.py tests/test_gpu_concurrent.py \
  "tests/test_gpu_parity.py::test_word_alignment_matrix_micro" "tests/test_gpu_parity.py::test_greedy_transcribe_matches_oracle" \
  tests/test_gpu_mx8.py tests/test_gpu_rccl.py tests/test_gpu_wide.py > $O/new_tests.log 2>&1
rc2=$?; tail -3 $O/new_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream > $O/bench_bf16.json 2> $O/bench_bf16.err
echo "bf16 bench rc $?"; head -c 300 $O/bench_bf16.json; echo
timeout -k 10 300 python bench.py --dtype f16 --steps 5 --no-cpu-baseline --no-stream > $O/bench_f16.json 2> $O/bench_f16.err
echo "f16 bench rc $?"; head -c 300 $O/bench_f16.json; echo
exit $((rc1 + rc2))
