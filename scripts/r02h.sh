set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_msk.py $R/tests/test_golden.py $R/tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['timed_region'])"
