#!/bin/bash
# final check at HEAD: the round-end GPU suite and smoke()
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03z
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
