#!/bin/bash
# Round-6 final verification (GPU box, repo root): every -m gpu test file but the step file, then the round profile
# (tools/profile_round.sh) with a heartbeat; sequential, the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r06_gpu.sh "${1:?tag}" tests1 || exit 1
(while sleep 50; do date >> gpurun_out/hb.txt; done) &
HB=$!
trap "kill $HB" EXIT
bash tools/profile_round.sh "${2:?profile tag}"
