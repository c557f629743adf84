#!/bin/bash
# Round-4 GPU check (b): C2 parity of the default build, A/B bench of the
# demod hand-off variants, MSK rate change (engine + host), the untraced
# burst scale test, then the demod diagnosis.
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $OUT/pytest_parity.log 2>&1
bash scripts/ab_bench.sh $TAG "r3 syncv1 base" --steps 10 --warmup 2 --h2d-steps 0 > $OUT/ab.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_msk_rate.py tests/test_gpu_msk.py "tests/test_gpu_host.py::test_msk_vfo_at_explicit_out_rate" > $OUT/pytest_msk.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_burst_scale.py > $OUT/pytest_burst_scale.log 2>&1
bash scripts/gpu_diag_demod.sh $TAG
