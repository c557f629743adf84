#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the burst
# kernels at the C4 bench config.
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex 'front_burst|demod_burst|hilbert|trident_kernel' --output-format csv \
    -d /tmp/pmcb_${TAG}_$c -o pmc -- python3 $R/bench.py --mode burst10500 --steps 3 --no-cpu-baseline > $OUT/pmc_$c.log 2>&1
  find /tmp/pmcb_${TAG}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$c.csv \;
done
ls -la $OUT
