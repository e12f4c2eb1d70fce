set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r02x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3 4; do
  rm -rf /tmp/sm$i
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sm$i -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-stream --steps 3 > $O/bench$i.log 2>&1 || exit 1
  KT=$(find /tmp/sm$i -name "run_kernel_trace.csv" -print -quit)
  python3 $R/tools/gap_stats.py "$KT" > $O/gaps$i.txt || exit 1
  rm -rf /tmp/sm$i
done
