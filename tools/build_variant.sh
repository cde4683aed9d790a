#!/usr/bin/env bash
# Builds an A/B variant of libmccs_hip.so with extra -D flags into exp/<name>.so
# (use it with MCCS_LIB_PATH=exp/<name>.so).  Only ring.hip is recompiled.
#   tools/build_variant.sh <name> -DMCCS_RING_INPUT_NT=1 ...
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/exp/$name"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -I"$R/mccs_amd/csrc" "$@" \
  -c -x hip "$R/mccs_amd/csrc/ring.hip" -o "$R/exp/$name/ring.o"
objs=$(ls "$R"/build/obj/*.o | grep -v '/ring.hip.o$')
hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/exp/$name.so" "$R/exp/$name/ring.o" $objs -lpthread
rm -rf "$R/exp/$name"
echo "$R/exp/$name.so"
