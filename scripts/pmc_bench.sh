#!/bin/bash
# GPU-box counter recipe: one rocprofv3 --pmc pass per counter group (never
# combined with runtime/sys traces), restricted to the engine's kernels.
# Usage: bash scripts/pmc_bench.sh TAG [bench args...]
set -eo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KRE='demod_oqpsk|coarse_kernel|frame_kernel|viterbi_kernel'
pass() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" --output-format csv \
    -d /tmp/pmc_${TAG}_${name} -o pmc -- python3 $R/bench.py $BENCH_ARGS --no-cpu-baseline > $OUT/$name.log 2>&1
  find /tmp/pmc_${TAG}_${name} -name '*counter_collection.csv' -exec cp {} $OUT/$name.csv \;
}
BENCH_ARGS="$*"
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass fetch FETCH_SIZE
pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
pass sq2 SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
ls -la $OUT
