#!/bin/bash
# atan2 / log table rows loaded where their index is known, held there by a
# scheduling barrier (variant ih): parity of every mode, then the A/B of C2,
# C4, burst MSK and C3.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4x
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_ih.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_math.py tests/test_gpu_parity.py tests/test_gpu_events.py tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_burst.py tests/test_gpu_burst_msk.py > $OUT/pytest.log 2>&1 || exit $?
bash scripts/ab_bench.sh r4x/c2 "base ih base ih" --steps 10 --warmup 3 > $OUT/ab_c2.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r4x/oq "base ih base ih" --mode burst10500 --steps 6 --warmup 2 > $OUT/ab_oq.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r4x/msk "base ih base ih" --mode burstmsk1200 --steps 6 --warmup 2 > $OUT/ab_msk.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r4x/c3 "base ih base ih" --mode msk600 --steps 20 --warmup 3 > $OUT/ab_c3.txt 2>&1
