#!/bin/bash
# OQPSK coarse ring of mixed samples (variant xr): continuous parity incl.
# the full-scale sample, then the C2 A/B against the base build.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4r
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_xr.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_events.py tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_pinned_push.py tests/test_gpu_fullscale.py > $OUT/pytest.log 2>&1 || exit $?
bash scripts/ab_bench.sh r4r/ab "base xr base xr" --steps 10 --warmup 3 > $OUT/ab.txt 2>&1
