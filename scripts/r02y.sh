#!/bin/bash
# Viterbi placement with the faster trellis step: beside scatter+demod (base), serial on the main stream (vitser), none (novit)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02y
mkdir -p $OUT
for v in base vitser novit base; do
  if [ "$v" = base ]; then so=$R/aero-cli_amd/libaero_engine.so; else so=$R/aero-cli_amd/libaero_engine_$v.so; fi
  AERO_ENGINE_SO=$so timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --steps 10 > $OUT/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep '^{' $OUT/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step"], d["timed_region"]["acars_items"])')"
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
