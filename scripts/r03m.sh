#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03m
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_msk.py $R/tests/test_gpu_c5.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 $R/bench.py --mode msk600 --steps 20 --no-cpu-baseline > $OUT/bench_msk600.log 2>&1
tail -1 $OUT/bench_msk600.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_ms_per_step"])'
