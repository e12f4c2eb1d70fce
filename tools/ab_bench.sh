#!/bin/bash
# Interleaved A/B of library builds on the default bench line (run on the GPU box from the repo root):
#   bash tools/ab_bench.sh <tag> <rounds> <name>...   (name "base" = wmx/libwmx.so, else wmx/libwmx_<name>.so from
#   tools/build_variant.sh; "name@VAR=VAL" runs it with one documented bench knob set); prints value, decode stage and the cross-attention / reduce_ln kernel figures per run.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:?tag}; R=${2:?rounds}; shift 2
mkdir -p "$O"
(while sleep 50; do date >> "$O/heartbeat.txt"; done) &
HB=$!
trap "kill $HB" EXIT
for r in $(seq 1 "$R"); do
  for spec in "$@"; do
    n=${spec%%@*}; kv=""; [ "$spec" = "$n" ] || kv=${spec#*@}
    lib=$PWD/realtime-whisper-asr_amd/wmx/libwmx.so
    [ "$n" = base ] || lib=$PWD/realtime-whisper-asr_amd/wmx/libwmx_$n.so
    n=${spec//[@=]/_}
    env WMX_LIB=$lib $kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-stream > "$O/${n}_$r.json" 2> "$O/${n}_$r.err" \
      || { echo "$n round $r failed"; exit 1; }
    python - "$O/${n}_$r.json" "$n" "$r" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>8} r{sys.argv[3]} value {d['value']:.1f} decode_ms {d['stage_ms'][5]:.2f} "
      f"enc_mfma {d['encoder']['isolated_gpu_batch']['mfma_util']:.3f} logmel_us {d['logmel']['us']} "
      f"mode {d['decode_mode']['mode']} layer_e2e_us {d['roofline'].get('layer_e2e_us')}", flush=True)
EOF
  done
done
