#!/bin/bash
# burst parity after batching the channels' initial-state upload
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02q
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_burst.py test_gpu_burst_msk.py \
  > $R/gpurun_out/r02q/pytest.log 2>&1
