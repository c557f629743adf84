#!/bin/bash
# Attribution of the OQPSK demod's HBM traffic, buffer by buffer: FETCH_SIZE
# and WRITE_SIZE (one rocprofv3 --pmc pass each) of demod_oqpsk_kernel at the
# bench configuration for the product build and for diagnostic builds that
# leave out one buffer's accesses (AERO_X_DROP, demod_oqpsk.hip).
# Usage: bash scripts/pmc_demod_buffers.sh TAG   (builds: aero-cli_amd/build.py drop variants)
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base drop1 drop2 drop4 drop8; do
  so=$R/aero-cli_amd/libaero_engine.so
  [ $v != base ] && so=$R/aero-cli_amd/libaero_engine_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    AERO_ENGINE_SO=$so timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk' --output-format csv \
      -d /tmp/pmcd_${TAG}_${v}_$c -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --h2d-steps 0 \
      > $OUT/pmcd_${v}_$c.log 2>&1
    rc=$?  # 1-3: bench checks (a drop build decodes nothing), not a fault
    [ $rc -ge 4 ] && exit $rc
    find /tmp/pmcd_${TAG}_${v}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmcd_${v}_$c.csv \;
  done
done
ls -la $OUT
