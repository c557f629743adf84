#!/bin/bash
# headline bench with the final-drain time (drain_ms), two runs, and 10/40-step runs
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ac
mkdir -p $OUT
cd $R
for k in 20 20 10 40; do
  timeout -k 10 400 python3 bench.py --steps $k --warmup 5 --no-cpu-baseline > $OUT/bench_$k.log 2>&1
  grep '^{' $OUT/bench_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["steps"], d["value"], d["ms_per_step"], d["drain_ms"], d["kernel_ms_per_step"], d["host_ms_per_step"])'
done
