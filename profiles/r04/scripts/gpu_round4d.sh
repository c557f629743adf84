#!/bin/bash
# Round-4 GPU check (d): untraced burst scale test, demod diagnosis, A/B.
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_burst_scale.py > $OUT/pytest_burst_scale.log 2>&1 || true
bash scripts/ab_bench.sh $TAG "${VARS:-base}" --steps 10 --warmup 2 --h2d-steps 0 > $OUT/ab.txt 2>&1
bash scripts/gpu_diag_demod.sh $TAG
