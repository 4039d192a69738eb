#!/bin/bash
# Build libwce.so variants with compile-time switches into build_variants/<name>/.
# usage: tools/variants.sh name1 "-DFLAG ..." [name2 "-D..."] ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=$ROOT/build_variants/$name
  mkdir -p "$out/obj"
  make -s -C "$ROOT/80211parallelestimation_amd/csrc" OUT="$out/libwce.so" B="$out/obj" \
       HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wall -Wno-unused-function $flags" "$out/libwce.so"
  echo "built $name: $flags"
done
