#!/bin/bash
# atan2 fast path with the quadrant folded into the table and fused Horner series: device math + parity, then A/B
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02af
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_math.py test_gpu_parity.py \
  > $R/gpurun_out/r02af/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02af "base oldatan base oldatan" --steps 10
