#!/bin/bash
# build_variant.sh NAME [FILE=SUBSTITUTE ...] [-DFLAG ...]: build libgsr into
# build/variants/libgsr_NAME.so through csrc/Makefile, optionally with csrc files replaced by
# other copies (e.g. render.hip=/tmp/render_old.hip) and extra compiler flags, for
# tools/gpu_abv.sh / tools/ab_kstats.sh.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
P=3d_gaussian_magic_change-segment_3dgs_amd
C=$P/csrc
declare -A sub
flags=()
for a in "$@"; do
  case $a in
    -*) flags+=("$a") ;;
    *=*) sub[${a%%=*}]=${a#*=} ;;
    *) flags+=("$a") ;;
  esac
done
src=$C
if [ ${#sub[@]} -gt 0 ]; then  # a sibling copy, so that the relative include paths still resolve
  src=$P/.variant_csrc
  rm -rf $src; cp -r $C $src
  for f in "${!sub[@]}"; do cp "${sub[$f]}" $src/$f; done
fi
mkdir -p build/variants
base="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wall -Wno-unused-function -Wno-unused-variable -fno-slp-vectorize"
make -s -j8 -C $src OUT=$PWD/build/variants/libgsr_$name.so OBJDIR=$PWD/build/variants/obj_$name \
  HIPFLAGS="$base ${flags[*]}"
[ "$src" = "$C" ] || rm -rf $src
rm -rf build/variants/obj_$name
echo built build/variants/libgsr_$name.so
