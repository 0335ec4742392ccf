#!/bin/bash
# Build a library variant variants/lib_<name>.so with extra defines (CPU container):
#   bash tools/build_variant.sh <name> [defines...]
# Loaded by tests / bench through KELPIE_HIP_LIB=$PWD/variants/lib_<name>.so.
set -eo pipefail
name=$1; shift
mkdir -p build/var_$name variants
make -s $(ls kelpie_amd/csrc/*.cpp | sed 's#kelpie_amd/csrc/\(.*\)\.cpp#build/\1.cpp.o#')
for f in kelpie_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -Wno-unused-result -Iinclude -Xarch_host -mavx2 "$@" -c $f -o build/var_$name/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o variants/lib_$name.so build/var_$name/*.o \
  build/*.cpp.o
