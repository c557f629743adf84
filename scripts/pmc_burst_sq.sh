#!/bin/bash
# SQ issue/wait counters of the burst demods (one pass, 8 SQ counters) at the
# C4 and burst-MSK bench configs.  Usage: bash scripts/pmc_burst_sq.sh TAG [engine.so]
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
[ -n "$2" ] && export AERO_ENGINE_SO=$R/$2
cd /tmp && export TMPDIR=/tmp
for m in burst10500 burstmsk1200; do
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --kernel-include-regex 'demod_burst|demod_bmsk' --output-format csv \
    -d /tmp/pmcsq_${TAG}_$m -o pmc -- python3 $R/bench.py --mode $m --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_sq_$m.log 2>&1
  find /tmp/pmcsq_${TAG}_$m -name '*counter_collection.csv' -exec cp {} $OUT/pmc_sq_$m.csv \;
done
ls -la $OUT
