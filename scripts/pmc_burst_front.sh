#!/bin/bash
# HBM bytes of the burst front end, Hilbert stage and demod (FETCH_SIZE and
# WRITE_SIZE in separate passes) at the C4 bench config.
# Usage: bash scripts/pmc_burst_front.sh TAG
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex 'front_burst|hilbert|demod_burst' --output-format csv \
    -d /tmp/pmcbf_${TAG}_$c -o pmc -- python3 $R/bench.py --mode burst10500 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_burst_$c.log 2>&1
  find /tmp/pmcbf_${TAG}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_burst_$c.csv \;
done
ls -la $OUT
