#!/bin/bash
# A/B: the bench line of several engine builds (libaero_engine_<v>.so, built
# by aero-cli_amd/build.py build_engine(variant=...)) in one GPU session.
# Usage: bash scripts/ab_bench.sh TAG "v1 v2 ..." [bench args...]
set -eo pipefail
TAG=$1; VARS=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for v in $VARS; do
  if [ "$v" = base ]; then so=$R/aero-cli_amd/libaero_engine.so; else so=$R/aero-cli_amd/libaero_engine_$v.so; fi
  # a timing-only variant may decode nothing (bench then exits 1): keep its line
  AERO_ENGINE_SO=$so timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/$v.log 2>&1 || [ $? -eq 1 ]
  echo "$v $(tail -1 $OUT/$v.log | python3 $R/scripts/ab_line.py)"
done
