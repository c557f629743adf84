#!/bin/bash
# chained coarse transforms (no bit-reversal LDS passes): parity + A/B vs the previous kernel
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02o
cd $R/tests
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_parity.py test_golden.py \
  test_gpu_msk.py test_gpu_c5.py > $R/gpurun_out/r02o/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02o "base old" --steps 10
