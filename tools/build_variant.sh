#!/bin/bash
# build_variant.sh NAME [FILE=SUBSTITUTE ...] [-DFLAG ...]: build libgsr into
# build/variants/libgsr_NAME.so, optionally with csrc files replaced by other copies
# (e.g. render.hip=/tmp/render_old.hip) and extra compiler flags, for tools/bench_variants.sh.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=3d_gaussian_magic_change-segment_3dgs_amd/csrc
declare -A sub
flags=()
for a in "$@"; do
  case $a in
    -*) flags+=("$a") ;;
    *=*) sub[${a%%=*}]=${a#*=} ;;
    *) flags+=("$a") ;;
  esac
done
srcs=()
for f in api.hip preprocess.hip binning.hip binning_rows.hip render.hip train.hip knn.hip dp.hip; do
  if [ -n "${sub[$f]}" ]; then cp "${sub[$f]}" $C/.variant_$f; srcs+=($C/.variant_$f); else srcs+=($C/$f); fi
done
mkdir -p build/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -fno-slp-vectorize \
  -Wno-unused-function -Wno-unused-variable "${flags[@]}" -shared -o build/variants/libgsr_$name.so "${srcs[@]}"
rm -f $C/.variant_*
echo built build/variants/libgsr_$name.so
