#!/bin/bash
# round 5, GPU call 21: the 64-deep ring with unit 1 of K-tile t + 1 staged in phase 1 (l1) instead of phase 0 (l0),
# microbenchmark builds interleaved on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05y}
mkdir -p $O
for i in 1 2 3; do
  for v in l0 l1; do
    timeout -k 10 180 tools/mb_$v > $O/mb_${v}_$i.txt 2>&1 || { echo "mb_$v failed"; tail -5 $O/mb_${v}_$i.txt; exit 1; }
    grep -E "MISMATCH|FAIL" $O/mb_${v}_$i.txt && exit 1
  done
done
python3 - "$O" <<'PY'
import re,sys,collections
O=sys.argv[1]; res=collections.defaultdict(lambda: collections.defaultdict(list))
for v in ['l0','l1']:
    for i in (1,2,3):
        for l in open(f'{O}/mb_{v}_{i}.txt'):
            m=re.match(r'(\w+)\s+M=.*?256x256\s+([\d.]+) us',l)
            if m: res[v][m.group(1)].append(float(m.group(2)))
for sh in ['qkv','out','fc1','fc2','conv2','xkv','sq4k']:
    print(sh, '  '.join(f"{v} {min(res[v][sh]):.1f}-{max(res[v][sh]):.1f}" for v in ['l0','l1']))
PY
exit 0
