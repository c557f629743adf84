set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_burst.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_burst.log 2>&1
timeout -k 10 400 python3 $R/bench.py --mode c5 --steps 20 > $OUT/bench_c5.log 2>&1
tail -1 $OUT/bench_c5.log | cut -c1-1500
timeout -k 10 600 python3 $R/bench.py --mode burst10500 --channels 16384 --steps 10 > $OUT/bench_burst.log 2>&1
tail -1 $OUT/bench_burst.log | cut -c1-2000
