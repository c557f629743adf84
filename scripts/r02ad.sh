#!/bin/bash
# burst MSK demod: 40 of the 80 matched-filter partial sums in registers (4 waves per CU) vs all in LDS (2 waves per CU)
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02ad
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_burst_msk.py \
  > $R/gpurun_out/r02ad/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02ad "base bmsk80" --mode burstmsk1200 --steps 4
