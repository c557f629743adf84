#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03w
mkdir -p $OUT
for v in nopa nopb; do
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_$v.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "matches_oracle" > $OUT/$v.log 2>&1; echo "$v $(tail -1 $OUT/$v.log)"
done
