#!/bin/bash
# Demod diagnosis on one box: per-section stamps of the chain wave
# (AERO_X_STAMPS build) and one SQ counter pass per group over the bench.
# Usage: bash scripts/gpu_diag_demod.sh TAG
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_stamps.so timeout -k 10 300 python scripts/demod_stamps.py 65536 > $OUT/stamps.log 2>&1
cd /tmp && export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA"; do
  n=$(echo $grp | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex 'demod_oqpsk' --output-format csv \
    -d /tmp/pmc_${TAG}_$n -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --h2d-steps 0 > $OUT/pmc_$n.log 2>&1
  find /tmp/pmc_${TAG}_$n -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$n.csv \;
done
cd $R

