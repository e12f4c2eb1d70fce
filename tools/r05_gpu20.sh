#!/bin/bash
# round 5, GPU call 20: the encoder attention's launch form on the half-tile-ring build (WMX_ENC_ATTN: default 8
# waves at <= 128 VGPRs, two workgroups per CU; 82: 8 waves at <= 256 VGPRs, one per CU; 4: 4-wave workgroups),
# interleaved default bench lines
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05v}
mkdir -p $O
for i in 1 2 3; do
  for v in 8 82 4; do
    WMX_ENC_ATTN=$v timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream > $O/b${i}_$v.json 2> $O/b${i}_$v.err || { echo "bench failed"; tail -5 $O/b${i}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b${i}_$v.json'));e=d['encoder'];g=e['isolated_gpu_batch'];print('b${i}_$v', d['value'], 'enc8', g['ms'], g['mfma_util'], 'insitu', e['insitu_stage_ms'])"
  done
done
exit 0
