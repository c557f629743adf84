#!/bin/bash
# LDS / VALU counter pass on the coarse FFT kernel (one rocprofv3 --pmc run
# per counter group).  Usage: bash scripts/pmc_coarse.sh TAG
set -eo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex 'coarse_kernel|demod_oqpsk' --output-format csv \
    -d /tmp/pmcc_${TAG}_${name} -o pmc -- python3 $R/bench.py --steps 3 --warmup 6 --channels 16384 --no-cpu-baseline > $OUT/$name.log 2>&1
  find /tmp/pmcc_${TAG}_${name} -name '*counter_collection.csv' -exec cp {} $OUT/$name.csv \;
}
pass lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVES SQ_INST_CYCLES_VMEM_RD
ls -la $OUT
