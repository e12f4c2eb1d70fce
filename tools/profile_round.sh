# Profile refresh for one round (run on the GPU box from the repo root):  bash tools/profile_round.sh r02a
# 1. HBM traffic of the decode-step kernels (separate rocprofv3 --pmc passes, tools/pmc_traffic.py)
#    -> profiles/<round>_pmc_traffic.json (the round = the tag without its letter suffix, e.g. r02)
# 2. the default bench line (which reports that traffic)
# 3. the same bench (no CPU baseline / streaming lines) under rocprofv3 --kernel-trace --stats: kernel / domain
#    summaries, the roofline recomputed from the trace (tools/roofline_from_profile.py), the post-decode stage
#    breakdown and the per-queue launch gaps.  The trace itself stays in /tmp (too large to merge back).
set -o pipefail
TAG=${1:?round tag, e.g. r02a}
ROUND=${TAG%[a-z]}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python "$R/tools/pmc_traffic.py" dec_qkv dec_proj dec_fc1 dec_fc2 reduce_ln cross_attn --batch 4 \
  --out "$O/pmc_traffic.json" > "$O/pmc.log" 2>&1 || exit 1
cp "$O/pmc_traffic.json" "$R/profiles/${ROUND}_pmc_traffic.json" || exit 1
timeout -k 10 400 python "$R/bench.py" > "$O/bench_default.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_$TAG
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-stream > "$O/bench_rocprof.log" 2>&1 || exit 1
KS=$(find /tmp/prof_$TAG -name "run_kernel_stats.csv" -print -quit)
DS=$(find /tmp/prof_$TAG -name "run_domain_stats.csv" -print -quit)
KT=$(find /tmp/prof_$TAG -name "run_kernel_trace.csv" -print -quit)
cp "$KS" "$O/kernel_stats.csv" && cp "$DS" "$O/domain_stats.csv" || exit 1
python3 "$R/tools/roofline_from_profile.py" "$KT" > "$O/roofline_from_trace.json" || exit 1
python3 "$R/tools/stage_kernels.py" "$KT" > "$O/align_stage.txt" || exit 1
python3 "$R/tools/gap_stats.py" "$KT" > "$O/gaps.txt" || exit 1
