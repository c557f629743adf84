#!/bin/bash
# burst OQPSK: 64-channel workgroups, RRC partial sums split registers / LDS (4 waves per CU)
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02t
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_burst.py \
  > $R/gpurun_out/r02t/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02t "base old" --mode burst10500 --steps 4
