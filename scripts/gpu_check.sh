#!/bin/bash
# One GPU call: the GPU suite (or a subset: $2 = pytest -k expression),
# smoke(), the default bench line and, with $3 = all, the other bench modes.
# Usage: bash scripts/gpu_check.sh TAG [K_EXPR] [all]
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu "${K[@]}" tests > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
if [ "$3" = all ]; then
  for m in burst10500 burstmsk1200 msk600 msk1200; do
    timeout -k 10 400 python bench.py --mode $m --steps 6 --cpu-runs 1 > $OUT/bench_$m.log 2>&1 || exit $?
  done
  timeout -k 10 300 python bench.py --mode c5 --steps 20 > $OUT/bench_c5.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --mode c1 > $OUT/bench_c1.log 2>&1 || exit $?
fi
