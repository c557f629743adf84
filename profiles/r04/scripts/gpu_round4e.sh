#!/bin/bash
# Round-4 GPU check (e): C2 parity of the default build, A/B, stamps.
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $OUT/pytest_parity.log 2>&1
bash scripts/ab_bench.sh $TAG "${VARS:-base}" --steps 10 --warmup 2 --h2d-steps 0 > $OUT/ab.txt 2>&1
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_stamps.so timeout -k 10 300 python scripts/demod_stamps.py 65536 > $OUT/stamps.log 2>&1
