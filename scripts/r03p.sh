#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03p
mkdir -p $OUT
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_corun.so timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash $R/scripts/ab_bench.sh r03p "base q16 corun" --steps 20 --warmup 5
