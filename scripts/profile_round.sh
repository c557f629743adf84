#!/bin/bash
# Round evidence on one GPU box, in three parts (each within one gpurun call).
#  part a: the headline bench line under the driver's own command, rocprofv3
#    kernel stats of that command, PMC HBM traffic of the demod and coarse
#    kernels at the bench config (FETCH_SIZE and WRITE_SIZE in separate
#    passes, MI355X_MICROARCH.md §HBM), SQ issue/wait counters of the same
#    kernels (one pass, 8 SQ counters).
#  part b: the burst (C4) and burst MSK (f1) lines with their kernel stats;
#  part c: C3 (msk600, msk1200), C5 in process with kernel stats, C5 through
#    the binaries, C1.
# Usage: bash scripts/profile_round.sh TAG a|b|c
set -eo pipefail
TAG=$1
PART=${2:-a}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "$PART" = a ]; then
  timeout -k 10 480 python3 $R/bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
  timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.log 2>&1
  find /tmp/prof_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk|coarse_kernel' --output-format csv \
      -d /tmp/pmc_${TAG}_$c -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --h2d-steps 0 > $OUT/pmc_$c.log 2>&1
    find /tmp/pmc_${TAG}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$c.csv \;
  done
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    --kernel-include-regex 'demod_oqpsk|coarse_kernel|viterbi_kernel' --output-format csv \
    -d /tmp/pmc_${TAG}_sq -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --h2d-steps 0 > $OUT/pmc_sq.log 2>&1
  find /tmp/pmc_${TAG}_sq -name '*counter_collection.csv' -exec cp {} $OUT/pmc_sq.csv \;
  python3 $R/tools/pmc_json.py $OUT/pmc_FETCH_SIZE.csv $OUT/pmc_WRITE_SIZE.csv $OUT/pmc_oqpsk10500.json oqpsk10500 65536 \
    "rocprofv3 --pmc, one pass per counter, bench.py --steps 4 --warmup 1 (65536 channels, after the 48-hop pre-roll; averages over every dispatch of the run), profiles/$TAG/pmc_{FETCH,WRITE}_SIZE.csv" > /dev/null
elif [ "$PART" = b ]; then
  timeout -k 10 600 python3 $R/bench.py --mode burst10500 --steps 10 --cpu-runs 1 > $OUT/bench_burst.log 2>&1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profb_$TAG -o prof -- python3 $R/bench.py --mode burst10500 --steps 6 --no-cpu-baseline > $OUT/bench_burst_prof.log 2>&1
  find /tmp/profb_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burst.csv \;
  timeout -k 10 600 python3 $R/bench.py --mode burstmsk1200 --steps 6 --cpu-runs 1 > $OUT/bench_burstmsk.log 2>&1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profm_$TAG -o prof -- python3 $R/bench.py --mode burstmsk1200 --steps 4 --no-cpu-baseline > $OUT/bench_burstmsk_prof.log 2>&1
  find /tmp/profm_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burstmsk.csv \;
else
  timeout -k 10 400 python3 $R/bench.py --mode msk600 --steps 20 --cpu-runs 1 > $OUT/bench_msk600.log 2>&1
  timeout -k 10 400 python3 $R/bench.py --mode msk1200 --steps 20 --cpu-runs 1 > $OUT/bench_msk1200.log 2>&1
  timeout -k 10 400 python3 $R/bench.py --mode c5 --steps 20 > $OUT/bench_c5.log 2>&1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc_$TAG -o prof -- python3 $R/bench.py --mode c5 --steps 20 --no-cpu-baseline > $OUT/bench_c5_prof.log 2>&1
  find /tmp/profc_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_c5.csv \;
  timeout -k 10 400 python3 $R/bench.py --mode c5bin --steps 3 > $OUT/bench_c5bin.log 2>&1
  timeout -k 10 400 python3 $R/bench.py --mode c1 > $OUT/bench_c1.log 2>&1
fi
ls -la $OUT
