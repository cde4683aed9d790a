#!/usr/bin/env bash
# Builds an A/B variant of libmccs_hip.so with extra -D flags into
# $VARIANT_DIR/<name>.so (default abvar/: git-ignored, but it travels to the
# GPU box; use it with MCCS_LIB_PATH=abvar/<name>.so).  Only the ring translation units
# (ring.hip, ring_ar_*.hip) are recompiled, in parallel; VARIANT_SRCS=reduce
# recompiles reduce.hip instead.
#   tools/build_variant.sh <name> -DMCCS_RING_INPUT_NT=1 ...
#   VARIANT_SRCS=reduce tools/build_variant.sh rtrace -DMCCS_REDUCE_TRACE
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
OUT="$R/${VARIANT_DIR:-abvar}"
mkdir -p "$OUT/$name"
pids=()
pat=${VARIANT_SRCS:-ring}
for src in "$R"/mccs_amd/csrc/$pat*.hip; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/include" -I"$R/mccs_amd/csrc" "$@" \
    -c -x hip "$src" -o "$OUT/$name/$(basename "$src").o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
objs=$(ls "$R"/build/obj/*.o | grep -v "/$pat[^/]*\.hip\.o\$")
hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/$name.so" "$OUT"/$name/*.o $objs -lpthread
rm -rf "$OUT/$name"
echo "$OUT/$name.so"
