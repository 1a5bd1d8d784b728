#!/bin/bash
# Build a variant of libblsverify.so with some kernel units recompiled under extra flags:
#   scripts/build_variant.sh NAME "k_miller.hip k_hash.hip" "-DBLS_WPE_LINES=1"  ->  variants/libblsverify_NAME.so
# (the other units are the current build/ objects). Load it with DRAND_AMD_LIB=variants/... .
set -e
name=$1; srcs=$2; flags=$3
cd "$(dirname "$0")/../drand_amd/csrc"
make -s ../libblsverify.so
mkdir -p ../../variants
d=build_$name
rm -rf $d && mkdir -p $d && cp build/*.o $d/
for src in $srcs; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -Wno-pass-failed $flags -c $src -o $d/${src%.hip}.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../variants/libblsverify_$name.so $d/*.o
rm -rf $d
echo variants/libblsverify_$name.so
