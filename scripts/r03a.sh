#!/bin/bash
# coarse-kernel section stamps at the bench config + the HEAD bench line
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03a
mkdir -p $OUT
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_stamps.so timeout -k 10 300 python3 -u $R/scripts/coarse_stamps.py 65536 > $OUT/coarse_stamps.log 2>&1
cat $OUT/coarse_stamps.log
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log
