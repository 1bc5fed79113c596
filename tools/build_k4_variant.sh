#!/bin/bash
# Link vct/libvct_hip_<name>.so from the current objects with vct_trace.hip compiled
# with extra flags (A/B of K4 build switches, tools/ab_libs_n.sh):
#   bash tools/build_k4_variant.sh <name> [-DVCT_K4_...=...]
set -e
cd "$(dirname "$0")/../voxel-based-global-illumination_amd"
name=$1; shift
make -j8 > /dev/null
H="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function"
mkdir -p build/var
/opt/rocm/bin/hipcc $H -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" -x hip -c csrc/vct_trace.hip -o build/var/vct_trace_$name.o
objs=$(ls build/obj/*.o | grep -v vct_trace.hip.o)
/opt/rocm/bin/hipcc $H -shared $objs build/var/vct_trace_$name.o -o vct/libvct_hip_$name.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
ls -la vct/libvct_hip_$name.so
