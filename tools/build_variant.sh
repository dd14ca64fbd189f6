#!/bin/bash
# Build an A/B variant of libdrt_hip.so: one source recompiled with extra -D flags, linked with the
# product objects of denseretrievaltoolkits_amd/build.  Load it with DRT_LIB=<path> (the product
# library and its ABI are unchanged).  Ablations live in a patched COPY of the source, never in the
# product source: SRC=<patched copy of csrc/<stem>.hip> (its #includes resolve against csrc/).
#   usage: [SRC=path] tools/build_variant.sh <name> <source stem, e.g. encoder> <flags...>
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; stem=$2; shift 2
B=$R/denseretrievaltoolkits_amd/build
V=$R/denseretrievaltoolkits_amd/variants
mkdir -p $V
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value -I$R/include \
  -I$R/denseretrievaltoolkits_amd/csrc "$@" -c ${SRC:-$R/denseretrievaltoolkits_amd/csrc/$stem.hip} -o $V/$stem.$name.o
objs=""
for o in $B/*.o; do
  if [ "$(basename $o)" = "$stem.o" ]; then objs="$objs $V/$stem.$name.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-soname,libdrt_hip.so $objs -o $V/libdrt_hip.$name.so
echo $V/libdrt_hip.$name.so
