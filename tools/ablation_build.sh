#!/bin/bash
# Debug-only timing builds (never the product): the WCE_ABLATE_* / WCE_LR_ABLATE_*
# blocks that skip a phase of a kernel (the back-substitution, the Ryy build,
# the tap DFTs, the lane kernel's loads or stores, the equalizer VALU) were
# retired from product source in round 5 (commit a856519).  That commit also
# rewrote ref_fc_kernel and changed the State layout, so a build of its parent
# is round 4's library, not the product: its timings cover only the ablated
# kernels, compared with the same parent built without the -D flags (never
# with the product).  This script exports the parent's WHOLE csrc tree
# (git archive a856519^) into build_variants/<name>/src and builds a
# libwce.so from it with the given -D flags, for the A/B tools
# (tools/ab_libs.py build_variants/<name> ...).
# usage: tools/ablation_build.sh name "-DWCE_ABLATE_BACKSOLVE -DWCE_ABLATE_KEEP=1"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; flags=$2
src=$ROOT/build_variants/$name/src
mkdir -p "$src" "$ROOT/build_variants/$name/obj"
git -C "$ROOT" archive a856519^ 80211parallelestimation_amd/csrc include | tar -x -C "$src" --strip-components=0
mv "$src"/80211parallelestimation_amd/csrc/* "$src/" && rm -rf "$src/80211parallelestimation_amd"
sed -i 's#\.\./\.\./include#'"$src"'/include#g; s#python3 \.\./srchash.py#true#' "$src/Makefile"
sed -i 's#"\.\./\.\./include/#"'"$src"'/include/#' "$src"/*.h "$src"/*.hip "$src"/*.cpp
make -s -C "$src" OUT="$ROOT/build_variants/$name/libwce.so" B="$ROOT/build_variants/$name/obj" \
     HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wall -Wno-unused-function $flags" \
     "$ROOT/build_variants/$name/libwce.so"
echo "built ablation $name: $flags (the whole csrc + include of a856519^; compare only with that parent built without flags)"
