#!/bin/bash
# round 3 (session 2), GPU call 37: the committed build (MX LayerNorm at one row per wave): MX-fp8 parity, the
# encoder parity tests and smoke
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03zy}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx8.py \
  tests/test_gpu_wide.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
tail -2 $O/smoke.log
