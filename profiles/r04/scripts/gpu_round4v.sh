#!/bin/bash
# OQPSK demod with time-major carrier / MSE rings (variant tm): continuous
# parity incl. the full-scale sample, the C2 A/B, the demod's HBM traffic.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4v
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_tm.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_events.py tests/test_gpu_pinned_push.py tests/test_gpu_fullscale.py > $OUT/pytest.log 2>&1 || exit $?
bash scripts/ab_bench.sh r4v/ab "base tm base tm" --steps 10 --warmup 3 > $OUT/ab.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for v in base tm; do
  so=$R/aero-cli_amd/libaero_engine_$v.so; [ $v = base ] && so=$R/aero-cli_amd/libaero_engine.so
  for c in FETCH_SIZE WRITE_SIZE; do
    AERO_ENGINE_SO=$so timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk' --output-format csv \
      -d /tmp/pmcv_${v}_$c -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --h2d-steps 0 > $OUT/pmc_${v}_$c.log 2>&1 || exit $?
    find /tmp/pmcv_${v}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_${v}_$c.csv \;
  done
done
