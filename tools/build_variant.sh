#!/bin/bash
# Link vct/libvct_hip_<name>.so from the current objects with ONE source recompiled with
# extra flags (A/B of build switches):
#   bash tools/build_variant.sh <name> <csrc file, e.g. vct_reorder.hip> [-DVCT_...=...]
set -e
cd "$(dirname "$0")/../voxel-based-global-illumination_amd"
name=$1; src=$2; shift 2
make -j8 > /dev/null
H="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function"
[ "$src" = vct_trace.hip ] && H="$H -mllvm -amdgpu-sched-strategy=iterative-ilp"
mkdir -p build/var
/opt/rocm/bin/hipcc $H "$@" -x hip -c csrc/$src -o build/var/${src}_$name.o
objs=$(ls build/obj/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc $H -shared $objs build/var/${src}_$name.o -o vct/libvct_hip_$name.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
ls -la vct/libvct_hip_$name.so
