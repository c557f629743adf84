#!/bin/bash
# two-rank union test, C1 end-to-end line, burst MSK bench line + kernel stats
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02p
mkdir -p $OUT
cd $R/tests
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread test_gpu_shard_union.py > $OUT/pytest_union.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --mode c1 > $OUT/bench_c1.log 2>&1
timeout -k 10 600 python3 $R/bench.py --mode burstmsk1200 --steps 6 > $OUT/bench_burstmsk.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profbm -o prof -- python3 $R/bench.py --mode burstmsk1200 --steps 4 --no-cpu-baseline > $OUT/bench_burstmsk_prof.log 2>&1
find /tmp/profbm -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burstmsk.csv \;
