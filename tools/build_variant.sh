#!/usr/bin/env bash
# Builds an A/B variant of libmccs_hip.so with extra -D flags into exp/<name>.so
# (use it with MCCS_LIB_PATH=exp/<name>.so).  Only the ring translation units
# (ring.hip, ring_ar_*.hip) are recompiled, in parallel; VARIANT_SRCS=reduce
# recompiles reduce.hip instead.
#   tools/build_variant.sh <name> -DMCCS_RING_INPUT_NT=1 ...
#   VARIANT_SRCS=reduce tools/build_variant.sh rtrace -DMCCS_REDUCE_TRACE
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/exp/$name"
pids=()
pat=${VARIANT_SRCS:-ring}
for src in "$R"/mccs_amd/csrc/$pat*.hip; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -I"$R/mccs_amd/csrc" "$@" \
    -c -x hip "$src" -o "$R/exp/$name/$(basename "$src").o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
objs=$(ls "$R"/build/obj/*.o | grep -v "/$pat[^/]*\.hip\.o\$")
hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/exp/$name.so" "$R"/exp/$name/*.o $objs -lpthread
rm -rf "$R/exp/$name"
echo "$R/exp/$name.so"
