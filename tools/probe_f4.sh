cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
{
echo "== nproc / affinity / cpu model"
nproc; python3 -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"
grep -m1 "model name" /proc/cpuinfo; lscpu | head -20
echo "== GL / EGL / OSMesa / llvmpipe libraries"
ldconfig -p | grep -iE "libEGL|OSMesa|libGL\.|gbm|swrast|llvmpipe|libGLX|vulkan|lvp" || echo "none via ldconfig"
find / -xdev \( -name "libEGL*.so*" -o -name "libOSMesa*" -o -name "*swrast_dri*" -o -name "libgbm*" -o -name "libvulkan_lvp*" -o -name "kms_swrast*" \) 2>/dev/null | head -40
echo "== glslang / glslangValidator"
which glslangValidator glslang glslc 2>&1 || true
} > gpurun_out/f4_probe.txt 2>&1
cat gpurun_out/f4_probe.txt | head -80
