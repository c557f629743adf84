set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02b
timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_msk.py $R/tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/r02b/pytest.log 2>&1
bash $R/scripts/ab_bench.sh r02b "base notriv ocml divmul" --steps 10
