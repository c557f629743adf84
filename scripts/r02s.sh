#!/bin/bash
# continuous MSK demod ring reads hoisted: parity + A/B (C3)
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02s
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_msk.py test_gpu_c5.py \
  > $R/gpurun_out/r02s/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02s "base old" --mode msk600 --steps 10
