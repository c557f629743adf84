#!/bin/bash
# round-3 evidence: full GPU suite, then the round profile (bench lines, rocprof stats, PMC traffic)
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash $R/scripts/profile_round.sh r03b
