#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03t
mkdir -p $OUT

timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_burst.py $R/tests/test_gpu_msk.py $R/tests/test_gpu_burst_msk.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_ms_per_step"])'
