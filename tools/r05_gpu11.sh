#!/bin/bash
# round 5, GPU call 11: per-launch breakdown of one encoder layer (bf16 and MX-fp8, rocprofv3 kernel trace of
# tools/encprof.py) on the half-tile rings, and the 16-window fp8 translate / bf16 lines
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05k}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
(while sleep 50; do date >> $O/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
for ct in bfloat16 float8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$ct -o run -- python3 tools/encprof.py $ct > $O/encprof_$ct.txt 2>&1 || { echo "encprof $ct failed"; tail -5 $O/encprof_$ct.txt; exit 1; }
  f=$(find $O/tr_$ct -name '*kernel_trace.csv' | head -1)
  python tools/enc_layer_breakdown.py $f > $O/layer_$ct.txt 2>&1; cat $O/layer_$ct.txt
  rm -f $f
done
timeout -k 10 300 python bench.py --dtype fp8 --task translate --batch 16 --steps 3 --no-cpu-baseline --no-stream \
  > $O/bench_fp8_b16.json 2> $O/bench_fp8_b16.err || { echo fp8 bench failed; tail -5 $O/bench_fp8_b16.err; exit 1; }
timeout -k 10 300 python bench.py --batch 16 --steps 3 --no-cpu-baseline --no-stream > $O/bench_bf16_b16.json \
  2> $O/bench_bf16_b16.err || { echo bf16 b16 bench failed; exit 1; }
for f in bench_fp8_b16 bench_bf16_b16; do python -c "import json;d=json.load(open('$O/$f.json'));e=d['encoder'];print('$f', d['value'], d['ms_per_step'], 'enc', e['isolated_ms'], e.get('isolated_mfma_util'), e.get('note'))"; done
exit 0
