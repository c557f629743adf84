#!/bin/bash
# GPU-box check at HEAD: the round-end GPU suite (or the tests named in
# $PYTEST_SEL) and smoke(), each under its own time limit.
# Usage: bash scripts/gpu_check.sh TAG
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-$R/tests} -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
