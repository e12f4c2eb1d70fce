#!/bin/bash
# round 5, GPU call 8: the encoder GEMM — in-kernel clock (s_memtime / s_memrealtime per tile), the 32-deep slice ring
# (cur) against the 64-deep half-tile ring (k64) interleaved on one box (each binary checks its 256 tile against the
# 128 tile), and L2-side request counts of both (one counter group per rocprofv3 pass)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05h}
mkdir -p $O
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
for v in st k64st; do
  timeout -k 10 180 tools/mb_gemm256_$v > $O/mb_$v.txt 2>&1 || { echo "mb_$v failed"; tail -5 $O/mb_$v.txt; exit 1; }
  echo "== $v"; grep -E "stamps|FAIL|MISMATCH" $O/mb_$v.txt
done
for i in 1 2 3; do
  for v in cur k64; do
    timeout -k 10 180 tools/mb_gemm256_$v > $O/mb_${v}_$i.txt 2>&1 || { echo "mb_$v failed"; tail -5 $O/mb_${v}_$i.txt; exit 1; }
    echo "== $v $i"; grep -E "^(qkv|out|fc1|fc2|sq4k)" $O/mb_${v}_$i.txt | awk '{print $1, $11, $12, $13, $14, $17}'
  done
done
for v in cur k64; do
for grp in "TCP_TCC_READ_REQ_sum TCC_REQ_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/pmc_${v}_$tag -o run --output-format csv -- tools/mb_gemm256_$v > $O/pmc_${v}_$tag.log 2>&1
  rc=$?; echo "pmc $v $tag rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
done
done
exit 0
