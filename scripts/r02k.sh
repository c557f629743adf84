#!/bin/bash
# burst MSK parity on the GPU, then the other burst tests
set -o pipefail
mkdir -p gpurun_out/r02k
cd tests
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread test_gpu_burst_msk.py \
  > ../gpurun_out/r02k/pytest_bmsk.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread test_gpu_burst.py \
  > ../gpurun_out/r02k/pytest_burst.log 2>&1
