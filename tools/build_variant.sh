#!/bin/bash
# Build the library with search.hip compiled under extra -D flags, for A/B
# runs (tools/ab_lib.sh, SAHARA_HIP_LIB): tools/build_variant.sh NAME -DFLAG ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p "$R/build/var" "$R/sahara_amd/lib/var"
make -C "$R" -s -j8 >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -c "$R/sahara_amd/csrc/search.hip" -o "$R/build/var/search_$N.o"
objs=$(ls "$R"/build/obj/*.o | grep -v '/search.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$R/build/var/search_$N.o" -o "$R/sahara_amd/lib/var/lib_$N.so" -lpthread
echo "$R/sahara_amd/lib/var/lib_$N.so"
