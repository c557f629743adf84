#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03g
mkdir -p $OUT
for v in stamps_head stamps_win; do
  AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_$v.so timeout -k 10 300 python3 -u $R/scripts/demod_stamps.py 65536 > $OUT/$v.log 2>&1
  echo "== $v"; cat $OUT/$v.log
done
