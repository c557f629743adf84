#!/bin/bash
# Viterbi trellis step: fixed column register per run, v_writelane, branch metric by sign (parity + A/B)
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02x
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_parity.py test_gpu_msk.py test_golden.py \
  > $R/gpurun_out/r02x/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02x "base oldvit" --steps 10
