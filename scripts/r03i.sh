#!/bin/bash
# demod/coarse HBM traffic (FETCH_SIZE, WRITE_SIZE: one rocprofv3 --pmc pass each) at the bench config
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk|coarse_kernel' --output-format csv \
    -d /tmp/pmc_r03i_$c -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/pmc_$c.log 2>&1
  find /tmp/pmc_r03i_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$c.csv \;
done
python3 $R/tools/pmc_summary.py $OUT/pmc_FETCH_SIZE.csv $OUT/pmc_WRITE_SIZE.csv
