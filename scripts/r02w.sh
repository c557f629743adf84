#!/bin/bash
# kernel + memory-copy timeline of the headline bench (base build), for the overlap analysis
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02w
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/tl -o tl -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1
find /tmp/tl -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
find /tmp/tl -name '*memory_copy_trace.csv' -exec cp {} $OUT/memory_copy_trace.csv \;
ls -la $OUT
