#!/bin/bash
# Debug-only timing builds (never the product): the WCE_ABLATE_* / WCE_LR_ABLATE_*
# blocks that skip a phase of a kernel (the back-substitution, the Ryy build,
# the tap DFTs, the lane kernel's loads or stores, the equalizer VALU) were
# retired from product source in round 5 (commit a856519, whose compiled
# device code is byte-identical to its parent's).  This script checks the
# parent's wce_kernels.hip out of git into build_variants/<name>/src and builds
# a libwce.so from it with the given -D flags, for the A/B tools
# (tools/ab_libs.py build_variants/<name> ...).
# usage: tools/ablation_build.sh name "-DWCE_ABLATE_BACKSOLVE -DWCE_ABLATE_KEEP=1"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; flags=$2
src=$ROOT/build_variants/$name/src
mkdir -p "$src" "$ROOT/build_variants/$name/obj"
cp "$ROOT"/80211parallelestimation_amd/csrc/* "$src/" 2>/dev/null || true
git -C "$ROOT" show a856519^:80211parallelestimation_amd/csrc/wce_kernels.hip > "$src/wce_kernels.hip"
git -C "$ROOT" show a856519^:80211parallelestimation_amd/csrc/wce_internal.h > "$src/wce_internal.h"
git -C "$ROOT" show a856519^:80211parallelestimation_amd/csrc/wce_api.cpp > "$src/wce_api.cpp"
git -C "$ROOT" show a856519^:80211parallelestimation_amd/csrc/wce_state.cpp > "$src/wce_state.cpp"
sed -i 's#\.\./\.\./include#'"$ROOT"'/include#g; s#python3 \.\./srchash.py#true#' "$src/Makefile"
sed -i 's#"\.\./\.\./include/#"'"$ROOT"'/include/#' "$src"/*.h "$src"/*.hip "$src"/*.cpp
make -s -C "$src" OUT="$ROOT/build_variants/$name/libwce.so" B="$ROOT/build_variants/$name/obj" \
     HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wall -Wno-unused-function $flags" \
     "$ROOT/build_variants/$name/libwce.so"
echo "built ablation $name: $flags (sources of a856519^)"
