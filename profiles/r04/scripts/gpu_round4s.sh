#!/bin/bash
# Coarse prologue loads issued with the state loads (pro), plus atan2 / log
# tables in LDS (tab): continuous parity of tab, then the C2 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4s
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_tab.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_events.py tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_math.py > $OUT/pytest.log 2>&1 || exit $?
bash scripts/ab_bench.sh r4s/ab "base pro tab base pro tab" --steps 10 --warmup 3 > $OUT/ab.txt 2>&1
