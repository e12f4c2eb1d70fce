#!/bin/bash
# round 5, GPU call 18: gemm256's tile order — 2, 4 (default) or 8 row panels walking the columns together inside an
# XCD's tile range (WMX_G256_GM), microbenchmark builds interleaved on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05t}
mkdir -p $O
for i in 1 2 3; do
  for v in g4 g2 g8; do
    timeout -k 10 180 tools/mb_$v > $O/mb_${v}_$i.txt 2>&1 || { echo "mb_$v failed"; tail -5 $O/mb_${v}_$i.txt; exit 1; }
    grep -E "MISMATCH|FAIL" $O/mb_${v}_$i.txt && exit 1
  done
done
python3 - "$O" <<'PY'
import re,sys,collections
O=sys.argv[1]; res=collections.defaultdict(lambda: collections.defaultdict(list))
for v in ['g4','g2','g8']:
    for i in (1,2,3):
        for l in open(f'{O}/mb_{v}_{i}.txt'):
            m=re.match(r'(\w+)\s+M=.*?256x256\s+([\d.]+) us',l)
            if m: res[v][m.group(1)].append(float(m.group(2)))
for sh in ['qkv','out','fc1','fc2','conv2','xkv','sq4k']:
    print(sh, '  '.join(f"{v} {min(res[v][sh]):.1f}-{max(res[v][sh]):.1f}" for v in ['g4','g2','g8']))
PY
exit 0
