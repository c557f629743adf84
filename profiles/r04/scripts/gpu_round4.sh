#!/bin/bash
# Round-4 GPU check: wave placement probe, C2 parity, A/B bench of engine
# builds, the new parity tests.  Usage: bash scripts/gpu_round4.sh TAG [variants]
set -eo pipefail
TAG=$1; VARS=${2:-"r3 base"}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 60 ./tools/wave_place > $OUT/wave_place.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $OUT/pytest_parity.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash scripts/ab_bench.sh $TAG "$VARS" --steps 10 --warmup 2 --h2d-steps 0 > $OUT/ab.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_pinned_push.py tests/test_gpu_burst_scale.py tests/test_gpu_fullscale.py > $OUT/pytest_new.log 2>&1
