set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
cat $OUT/bench.log | tail -1 | cut -c1-900
