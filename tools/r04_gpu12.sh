#!/bin/bash
# round 4, GPU call 12: PMC passes over the decode step's reduce_ln launch alone (4 windows x beam 5 = the 20 rows of
# one bench context group): wave-cycle split (busy / waiting / issuing), instruction mix, L2 behaviour
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r04r}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python tools/redln_pmc.py > $O/plain.log 2>&1 || { echo plain failed; tail -5 $O/plain.log; exit 1; }
cat $O/plain.log
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex reduce_ln --pmc $P --output-format csv -d $O/p$i -o pmc -- python3 tools/redln_pmc.py \
    > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python tools/pmc_summary.py $O reduce_ln | tee $O/summary.txt
exit 0
