#!/bin/bash
# Build a variant of libwmx.so with extra compile-time defines for A/B runs (e.g. the cache-policy switches in
# csrc/wmx_common.h):  bash tools/build_variant.sh <name> -DWMX_WNT=1 ...  ->  wmx/libwmx_<name>.so
# Select it at run time with WMX_LIB=<abs path> (wmx/_lib.py); objects go under build/variants/<name>/.
set -e
name=$1; shift
cd "$(dirname "$0")/../realtime-whisper-asr_amd"
out=build/variants/$name
mkdir -p "$out"
objs=""
for src in csrc/*.hip; do
  o=$out/$(basename "${src%.hip}").o
  extra=""; [ "$(basename "$src")" = wmx_logmel.hip ] && extra=-fno-slp-vectorize  # as the Makefile builds it
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $extra -w "$@" -c "$src" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "wmx/libwmx_$name.so" $objs -lpthread
echo "wmx/libwmx_$name.so"
