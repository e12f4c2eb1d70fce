#!/bin/bash
# round 4, GPU call 5: HBM traffic of the decode launches from rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE in
# separate passes, tools/pmc_traffic.py) at 4 and 8 windows per group, bf16 and the fp8 decode
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04i}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
rm -f profiles/r04_pmc_traffic.json
timeout -k 10 1100 python tools/pmc_traffic.py dec_qkv dec_proj dec_fc1 dec_fc2 cross_attn reduce_ln --batch 4 8 \
  --dtype bfloat16 float8 --out profiles/r04_pmc_traffic.json --work $O/pmc > $O/pmc.log 2>&1
rc=$?
cp profiles/r04_pmc_traffic.json $O/ 2>/dev/null
find $O/pmc -name '*.db' -delete 2>/dev/null
tail -30 $O/pmc.log
exit $rc
