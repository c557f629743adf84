#!/bin/bash
# SQ counters of the coarse and demod kernels at the bench config (one rocprofv3 --pmc pass per group)
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03y
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex 'coarse_kernel|demod_oqpsk|viterbi_kernel' --output-format csv \
    -d /tmp/pmcy_${name} -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1
  find /tmp/pmcy_${name} -name '*counter_collection.csv' -exec cp {} $OUT/$name.csv \;
}
pass lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA
python3 $R/tools/pmc_summary.py $OUT/lds.csv $OUT/wait.csv
