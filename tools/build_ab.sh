#!/bin/bash
# Build vct/libvct_hip_base.so from HEAD (stashing the working tree) and
# vct/libvct_hip.so from the working tree, for tools/ab_libs.sh.
set -e
cd "$(dirname "$0")/../voxel-based-global-illumination_amd"
git stash -q
trap 'git stash pop -q' EXIT
make -j8 > /dev/null
cp vct/libvct_hip.so vct/libvct_hip_base.so
git stash pop -q
trap - EXIT
touch csrc/*.hip csrc/*.cpp
make -j8 > /dev/null
ls -la vct/libvct_hip.so vct/libvct_hip_base.so
