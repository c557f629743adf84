#!/bin/bash
# OQPSK demod FIR: tap pairs outside-in sharing one product, taps from constant memory: parity, then A/B
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02ah
cd $R/tests
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_parity.py test_golden.py test_gpu_c5.py \
  > $R/gpurun_out/r02ah/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02ah "base oldfir base oldfir" --steps 10
