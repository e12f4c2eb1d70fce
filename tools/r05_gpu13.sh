#!/bin/bash
# round 5, GPU call 13: the direct epilogue on C^T fragments (MFMA operands swapped: a lane holds 4 consecutive
# columns of a row, no in-quad transpose) against the transposing epilogue, microbenchmark builds interleaved; the
# encoder GPU tests on the library build; interleaved bench lines against the transposing build (WMX_LIB)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05n}
mkdir -p $O
for i in 1 2 3; do
  for v in new noswap; do
    timeout -k 10 180 tools/mb_gemm256_$v > $O/mb_${v}_$i.txt 2>&1 || { echo "mb_$v failed"; tail -5 $O/mb_${v}_$i.txt; exit 1; }
    grep -E "MISMATCH|FAIL" $O/mb_${v}_$i.txt && exit 1
    echo "== $v $i"; grep -E "^(qkv|fc1|xkv|sq4k)" $O/mb_${v}_$i.txt | awk '{print $1, $11, $12, $13, $14, $15, $16, $17}'
  done
done
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_wide.py tests/test_gpu_mx8.py tests/test_gpu_step.py -k "full_depth or encoder or mx8 or wide or greedy or fold" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_swapall.so timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_step.py \
  -k "full_depth or encoder or wide or greedy or fold" > $O/tests_swapall.log 2>&1
rc=$?; tail -2 $O/tests_swapall.log
if [ $rc -ne 0 ]; then echo "swapall tests failed"; grep -E "FAILED|Error|assert" $O/tests_swapall.log | head -20; exit 1; fi
for i in 1 2 3; do
  for v in swap noswap swapall; do
    if [ $v != swap ]; then export WMX_LIB=$PWD/realtime-whisper-asr_amd/wmx/libwmx_$v.so; else unset WMX_LIB; fi
    timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_$v.json 2> $O/b${i}_$v.err || { echo "bench failed"; tail -5 $O/b${i}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_$v.json'));e=d['encoder'];g=e['isolated_gpu_batch'];print('b${i}_$v', d['value'], d['ms_per_step'], 'enc4', e['isolated_ms'], 'enc8', g['ms'], g['mfma_util'], 'insitu', e['insitu_stage_ms'])"
  done
done
unset WMX_LIB
exit 0
