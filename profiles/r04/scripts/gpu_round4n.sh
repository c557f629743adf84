#!/bin/bash
# Round-4 GPU check (n): MSK at 24 kHz with two imaginary partial sums in
# registers (two workgroups per CU): MSK parity, then MSK 1200 / C3 / C5 A/B.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT/m1200 $OUT/m600 $OUT/c5
cd $R
for v in base mskmc; do
  so=$R/aero-cli_amd/libaero_engine.so; [ $v = base ] || so=$R/aero-cli_amd/libaero_engine_$v.so
  AERO_ENGINE_SO=$so timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_c5.py > $OUT/pytest_$v.log 2>&1 || exit $?
done
bash scripts/ab_bench.sh $TAG/m1200 "mskold base msknolicm mskmc" --mode msk1200 --steps 10 > $OUT/ab_msk1200.txt 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG/m600 "mskold base mskmc" --mode msk600 --steps 10 > $OUT/ab_msk600.txt 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG/c5 "mskold base mskmc" --mode c5 --steps 20 > $OUT/ab_c5.txt 2>&1
