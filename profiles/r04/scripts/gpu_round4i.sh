#!/bin/bash
# Round-4 GPU check (i): the whole GPU suite (interleaved group passes,
# queued host pushes), C5 through the binaries, the C2 bench line.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --mode c5bin --steps 3 > $OUT/bench_c5bin.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --mode c5 --steps 3 > $OUT/bench_c5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1
