#!/bin/bash
# kernel timelines of the serial-Viterbi and no-Viterbi builds
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02z
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in vitser novit; do
  AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/tl_$v -o tl -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/bench_$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  find /tmp/tl_$v -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace_$v.csv \;
  find /tmp/tl_$v -name '*memory_copy_trace.csv' -exec cp {} $OUT/memory_copy_trace_$v.csv \;
done
ls -la $OUT
