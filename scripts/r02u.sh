#!/bin/bash
# A/B: Viterbi overlap cost (novit: job records only; vitser: decode on the main stream)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02u
mkdir -p $OUT
for v in base vitser novit; do
  if [ "$v" = base ]; then so=$R/aero-cli_amd/libaero_engine.so; else so=$R/aero-cli_amd/libaero_engine_$v.so; fi
  AERO_ENGINE_SO=$so timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --steps 10 > $OUT/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
