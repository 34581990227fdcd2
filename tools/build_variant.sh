#!/bin/bash
# Build libmirec.so with extra -D flags into recbole_amd/_lib/alt/<name>.so
# (profiling variants; the product library is recbole_amd/_lib/libmirec.so).
# usage: [PATCH=tools/patches/X.patch] tools/build_variant.sh NAME -DFLAG ...
# PATCH: a diff against recbole_amd/csrc applied to a scratch copy first (the probe
# builds that are kept out of the product sources, e.g. step_probes_r4.patch for the
# K35 stamps / hand-off variants; their full tree is branch probes/k35-r4).
set -eu
name=$1; shift
out=recbole_amd/_lib/alt
src=recbole_amd/csrc
mkdir -p $out /tmp/variant_$name
if [ -n "${PATCH:-}" ]; then
  t=/tmp/variant_src_$name                  # same depth as the tree: ../../include resolves
  rm -rf $t; mkdir -p $t/recbole_amd
  cp -r recbole_amd/csrc $t/recbole_amd/csrc
  rm -rf $t/recbole_amd/csrc/build
  ln -s "$PWD/include" $t/include
  (cd $t/recbole_amd/csrc && patch -p0 -s < "$OLDPWD/$PATCH")
  src=$t/recbole_amd/csrc
fi
rm -f /tmp/variant_$name/*.o
ls $src/*.hip | xargs -P 6 -I{} sh -c '/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC \
  --offload-arch=gfx950 -munsafe-fp-atomics -Iinclude -I'$src' '"$*"' -c {} \
  -o /tmp/variant_'$name'/$(basename {} .hip).o' || { echo "variant build failed"; exit 1; }
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/$name.so /tmp/variant_$name/*.o
echo built $out/$name.so
