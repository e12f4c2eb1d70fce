#!/bin/bash
# Build libwmx.so of an earlier git revision as wmx/libwmx_<name>.so, for interleaved A/B runs on one box
# (select it with WMX_LIB=<abs path>):  bash tools/build_rev.sh <name> <rev>
set -e
name=$1; rev=$2
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$root" archive "$rev" realtime-whisper-asr_amd/csrc include | tar -x -C "$tmp"
objs=""
for src in "$tmp"/realtime-whisper-asr_amd/csrc/*.hip; do
  o="$tmp/$(basename "${src%.hip}").o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -c "$src" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$root/realtime-whisper-asr_amd/wmx/libwmx_$name.so" $objs -lpthread
rm -rf "$tmp"
echo "realtime-whisper-asr_amd/wmx/libwmx_$name.so"
