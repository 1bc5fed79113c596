#!/bin/bash
# Copy the summaries of a tools/profile.sh run into profiles/ (tracked).
#   tools/collect_profiles.sh <tag> <round>   e.g. r1c r01
set -e
cd "$(dirname "$0")/.."
TAG=$1; RND=${2:-r01}
SRC=gpurun_out/prof_$TAG
mkdir -p profiles
cp $SRC/trace/trace_kernel_stats.csv profiles/${RND}_${TAG}_kernel_stats.csv
python3 tools/pmc_summary.py $SRC "${KSEL:-k4_trace}" > profiles/${RND}_${TAG}_k4_pmc.json
head -c 2000 $SRC/trace.stdout > profiles/${RND}_${TAG}_bench_under_rocprof.json || true
ls -la profiles/
