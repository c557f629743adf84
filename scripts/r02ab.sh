#!/bin/bash
# full GPU suite + smoke + headline bench after the Viterbi/push changes
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ab
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1
timeout -k 10 400 python3 bench.py --mode msk600 --steps 20 --no-cpu-baseline > $OUT/bench_msk600.log 2>&1
tail -1 $OUT/pytest.log; cat $OUT/smoke.log | tail -1
