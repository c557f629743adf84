#!/bin/bash
# burst demod ring reads hoisted ahead of the stores: parity, then burst OQPSK / MSK A/B
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02r
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_burst.py test_gpu_burst_msk.py \
  > $R/gpurun_out/r02r/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02r_boq "base old" --mode burst10500 --steps 4
bash $R/scripts/ab_bench.sh r02r_bmsk "base old" --mode burstmsk1200 --steps 4
