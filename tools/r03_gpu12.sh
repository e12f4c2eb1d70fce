#!/bin/bash
# round 3, GPU call 12: interleaved bench A/B of the current build against libwmx_base.so (the build before the
# alignment-tile / DTW / language-detect changes)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03t
mkdir -p $O
L=$PWD/realtime-whisper-asr_amd/wmx
for r in 1 2 3 4; do
  for v in base new; do
    if [ $v = base ]; then export WMX_LIB=$L/libwmx_base.so; else unset WMX_LIB; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $O/b.json 2> $O/b.err \
      || { echo "bench $v failed"; exit 1; }
    python - "$v" $O/b.json <<'PY' | tee -a $O/ab.txt
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:5s} {j['value']:8.2f}x {j['ms_per_step']:7.2f} ms stages {j['stage_ms']} mode {j['decode_mode']['mode']}")
PY
  done
done
