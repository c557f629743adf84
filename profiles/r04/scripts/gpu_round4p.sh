#!/bin/bash
# Round-4 GPU check (p): MSK parity at HEAD, the C3 line, the MSK 1200 line.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_c5.py tests/test_gpu_chan.py tests/test_gpu_host.py > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --mode msk600 --steps 20 --cpu-runs 1 > $OUT/bench_msk600.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --mode msk1200 --steps 20 --cpu-runs 1 > $OUT/bench_msk1200.log 2>&1
