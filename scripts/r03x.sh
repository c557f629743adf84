#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03x
mkdir -p $OUT
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_chunk.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "matches_oracle" > $OUT/chunk_parity.log 2>&1; echo "parity $(tail -1 $OUT/chunk_parity.log)"
bash $R/scripts/ab_bench.sh r03x "base chunk" --steps 10 --warmup 3
