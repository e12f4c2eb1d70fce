#!/bin/bash
# round 3, GPU call 10: column tiles per workgroup of the decode fc1 / fc2 (WMX_PACKED_NCT): the split form uses
# 160 workgroups for each (NCT 2 / 4), i.e. 160 of 256 CUs pull their weights; NCT 1 / 2 spread them over 320.
# Parity first (the teacher-forced step tests with both overrides), then an interleaved bench A/B.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03p
mkdir -p $O
export PYTHONUNBUFFERED=1
WMX_PACKED_NCT="5120:1280:4,1280:1280:4,3840:1280:4" timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -m gpu tests/test_gpu_step.py -k "forced_steps_wide or search_replay_wide" > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log
if [ $rc -ne 0 ]; then echo "parity with the NCT override failed (rc $rc): stopping"; exit 1; fi
for r in 1 2 3; do
  for v in "none" "5120:1280:4" "1280:1280:4" "3840:1280:4"; do
    WMX_PACKED_NCT="$v" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
      || { echo "bench $v failed"; exit 1; }
    python - "$v" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = j["roofline"]["layer_e2e_us"]
print(f"{sys.argv[1]:28s} {j['value']:8.2f}x decode {j['stage_ms'][5]:7.2f} ms mode {j['decode_mode']['mode']} "
      f"fc1 {e.get('dec_fc1')} fc2 {e.get('dec_fc2')} frac {j['roofline']['frac']}")
PY
  done
done
