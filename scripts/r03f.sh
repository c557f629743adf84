#!/bin/bash
# full GPU suite + bench line
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_ms_per_step"], d["timed_region"])'
