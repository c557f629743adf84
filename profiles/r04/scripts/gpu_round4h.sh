#!/bin/bash
# Round-4 GPU check (h): queued host pushes (parity, host binaries, full
# scale), C5 through the binaries, the C2 bench line.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -v -x --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_msk_rate.py tests/test_gpu_host.py tests/test_gpu_chan.py tests/test_gpu_c5.py tests/test_gpu_fullscale.py > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --mode c5bin --steps 3 > $OUT/bench_c5bin.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1
