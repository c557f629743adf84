#!/bin/bash
# GPU-box profiling recipe: bench line + rocprofv3 kernel-trace stats.
# Usage (from the repo root on the box): bash scripts/prof_bench.sh TAG [bench args...]
set -eo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 480 python3 $R/bench.py "$@" > $R/gpurun_out/$TAG/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py "$@" --no-cpu-baseline > $R/gpurun_out/$TAG/bench_prof.log 2>&1
find /tmp/prof_$TAG -name '*stats*.csv' -exec cp {} $R/gpurun_out/$TAG/ \;
find /tmp/prof_$TAG -name '*kernel_trace.csv' -exec sh -c 'grep -E "Kernel_Name|demod|coarse|frame_kernel|viterbi|scatter" "$1" > '$R'/gpurun_out/'$TAG'/aero_kernel_trace.csv' _ {} \;
ls -la $R/gpurun_out/$TAG
