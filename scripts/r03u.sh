#!/bin/bash
# the driver's round-end commands: smoke() then the default bench line
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03u
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_ms_per_step"], d["cpu_baseline"]["value"])'
