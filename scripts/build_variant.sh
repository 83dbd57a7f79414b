#!/bin/bash
# Build an A/B variant of libppo_hip.so: ppo_update.hip (or the file given) compiled with extra flags,
# linked with the other in-tree objects.   scripts/build_variant.sh <name> "<hipcc flags>" [update source]
set -e
NAME=$1; FLAGS=$2; SRC=${3:-csrc/ppo_update.hip}
cd "$(dirname "$0")/../ppo.cpp_amd"
make -s lib/libppo_hip.so
mkdir -p build_var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-pass-failed -Icsrc $FLAGS -c $SRC -o build_var/ppo_update_$NAME.o
OBJS=$(ls build/*.o | grep -v ppo_update.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/libppo_hip_$NAME.so $OBJS build_var/ppo_update_$NAME.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
ls -la lib/libppo_hip_$NAME.so
