#!/bin/bash
# sincos Ziv fast path: device math + parity (OQPSK, MSK, burst), then A/B
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02ag
cd $R/tests
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_math.py test_gpu_parity.py test_gpu_msk.py test_gpu_burst.py test_gpu_burst_msk.py \
  > $R/gpurun_out/r02ag/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02ag "base oldsc base oldsc" --steps 10
