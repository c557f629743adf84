#!/bin/bash
# Final check at HEAD, as the driver runs it: the GPU suite, smoke(), the
# default bench line.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1
