#!/bin/bash
# Build libmirec.so with extra -D flags into recbole_amd/_lib/alt/<name>.so
# (profiling variants; the product library is recbole_amd/_lib/libmirec.so).
# usage: tools/build_variant.sh NAME -DFLAG ...
set -eu
name=$1; shift
out=recbole_amd/_lib/alt
mkdir -p $out /tmp/variant_$name
for f in recbole_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics \
    -Iinclude "$@" -c $f -o /tmp/variant_$name/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/$name.so /tmp/variant_$name/*.o
echo built $out/$name.so
