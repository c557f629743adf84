#!/bin/bash
# Burst demods with event-aligned symbol steps (variant ev): burst parity,
# then the C4 and burst-MSK A/B against HEAD's burst code (variant pf).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4t
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_ev.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_burst.py tests/test_gpu_burst_msk.py tests/test_gpu_burst_scale.py > $OUT/pytest.log 2>&1 || exit $?
bash scripts/ab_bench.sh r4t/oq "pf ev pf ev" --mode burst10500 --steps 6 --warmup 2 > $OUT/ab_oq.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r4t/msk "pf ev pf ev" --mode burstmsk1200 --steps 6 --warmup 2 > $OUT/ab_msk.txt 2>&1
