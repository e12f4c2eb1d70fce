#!/bin/bash
# round 5, GPU call 10: the MX-fp8 256 GEMM on the 128-deep half-tile ring, and segment pinning (a scheduling
# barrier after each segment's opening s_barrier) for both GEMMs — microbenchmark builds interleaved on one box, then
# the MX-fp8 / parity GPU tests on the library build (new defaults)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05j}
mkdir -p $O
export PYTHONUNBUFFERED=1
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3; do
  for v in new nopin mx64; do
    timeout -k 10 180 tools/mb_gemm256_$v > $O/mb_${v}_$i.txt 2>&1 || { echo "mb_$v failed"; tail -5 $O/mb_${v}_$i.txt; exit 1; }
    echo "== $v $i"; grep -E "^(qkv|out|fc1|fc2|sq4k)" $O/mb_${v}_$i.txt | awk '{print $1, $12, $13, $14, $15, $21, $22, $23}'
  done
done
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread -m gpu tests/test_gpu_mx8.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; fi
exit 0
