#!/bin/bash
# One GPU session: parity tests, the headline bench line (the driver's own
# command) + rocprofv3 kernel stats of the same command, then extra bench
# modes.  Usage: bash scripts/gpu_session.sh TAG [modes...]
set -eo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
bash $R/scripts/prof_bench.sh $TAG --steps 20 --warmup 5
for m in "$@"; do
  timeout -k 10 480 python3 $R/bench.py --mode $m > $OUT/bench_$m.log 2>&1
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv \
     -d /tmp/prof_${TAG}_$m -o prof -- python3 $R/bench.py --mode $m --no-cpu-baseline > $OUT/bench_prof_$m.log 2>&1)
  find /tmp/prof_${TAG}_$m -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$m.csv \;
done
ls -la $OUT
