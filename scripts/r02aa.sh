#!/bin/bash
# device pushes straight into the PCM ring (high-priority side stream): parity of the push paths, then
# Viterbi beside the demod (base) vs serial (vitser), and a timeline of each
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02aa
mkdir -p $OUT
cd $R/tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread test_gpu_parity.py test_gpu_chan.py test_golden.py \
  > $OUT/pytest.log 2>&1 || exit 1
for v in base vitser base vitser; do
  if [ "$v" = base ]; then so=$R/aero-cli_amd/libaero_engine.so; else so=$R/aero-cli_amd/libaero_engine_$v.so; fi
  AERO_ENGINE_SO=$so timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --steps 20 > $OUT/$v.log 2>&1 || exit 1
  echo "$v $(grep '^{' $OUT/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms_per_step"], d["timed_region"]["acars_items"])')"
done
cd /tmp && export TMPDIR=/tmp
for v in base vitser; do
  if [ "$v" = base ]; then so=$R/aero-cli_amd/libaero_engine.so; else so=$R/aero-cli_amd/libaero_engine_$v.so; fi
  AERO_ENGINE_SO=$so timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/tl_$v -o tl -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/tl_$v.log 2>&1 || exit 1
  find /tmp/tl_$v -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace_$v.csv \;
done
