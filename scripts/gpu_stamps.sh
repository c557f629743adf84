#!/bin/bash
# Per-section cycle totals of the coarse kernel and the OQPSK demod chain wave
# (AERO_X_STAMPS build, aero-cli_amd/libaero_engine_stamps.so) at the bench
# configuration.  Usage: bash scripts/gpu_stamps.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_stamps.so
timeout -k 10 300 python -u scripts/coarse_stamps.py > $OUT/coarse_stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/demod_stamps.py > $OUT/demod_stamps.log 2>&1 || exit $?
