#!/bin/bash
# Round evidence on one GPU box: the headline bench line under the driver's
# own command, rocprofv3 kernel stats of that command, PMC HBM traffic of the
# demod kernel at the bench config (FETCH_SIZE and WRITE_SIZE in separate
# passes, MI355X_MICROARCH.md §HBM), then the burst (C4) and C5 lines with
# their kernel stats, C3 (msk600), burst MSK (f1) and the C1 end-to-end line.
# Usage: bash scripts/profile_round.sh TAG
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 python3 $R/bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.log 2>&1
find /tmp/prof_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk|coarse_kernel' --output-format csv \
    -d /tmp/pmc_${TAG}_$c -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/pmc_$c.log 2>&1
  find /tmp/pmc_${TAG}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$c.csv \;
done
python3 $R/tools/pmc_json.py $OUT/pmc_FETCH_SIZE.csv $OUT/pmc_WRITE_SIZE.csv $OUT/pmc_oqpsk10500.json oqpsk10500 65536 \
  "rocprofv3 --pmc, one pass per counter, bench.py --steps 4 --warmup 1 (65536 channels, after the 48-hop pre-roll; averages over every dispatch of the run), profiles/$TAG/pmc_{FETCH,WRITE}_SIZE.csv" > /dev/null
timeout -k 10 600 python3 $R/bench.py --mode burst10500 --steps 10 > $OUT/bench_burst.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profb_$TAG -o prof -- python3 $R/bench.py --mode burst10500 --steps 6 --no-cpu-baseline > $OUT/bench_burst_prof.log 2>&1
find /tmp/profb_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burst.csv \;
timeout -k 10 400 python3 $R/bench.py --mode c5 --steps 20 > $OUT/bench_c5.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profc_$TAG -o prof -- python3 $R/bench.py --mode c5 --steps 20 --no-cpu-baseline > $OUT/bench_c5_prof.log 2>&1
find /tmp/profc_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_c5.csv \;
timeout -k 10 400 python3 $R/bench.py --mode msk600 --steps 20 > $OUT/bench_msk600.log 2>&1
timeout -k 10 600 python3 $R/bench.py --mode burstmsk1200 --steps 6 > $OUT/bench_burstmsk.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profm_$TAG -o prof -- python3 $R/bench.py --mode burstmsk1200 --steps 4 --no-cpu-baseline > $OUT/bench_burstmsk_prof.log 2>&1
find /tmp/profm_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burstmsk.csv \;
timeout -k 10 400 python3 $R/bench.py --mode c1 > $OUT/bench_c1.log 2>&1
ls -la $OUT
