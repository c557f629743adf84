#!/bin/bash
# non-temporal PCM/AGC ring access: bench A/B + demod FETCH/WRITE counters per variant
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02m
mkdir -p $OUT
bash $R/scripts/ab_bench.sh r02m "base nt" --steps 10
cd /tmp && export TMPDIR=/tmp
for v in base nt; do
  if [ "$v" = base ]; then so=$R/aero-cli_amd/libaero_engine.so; else so=$R/aero-cli_amd/libaero_engine_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    AERO_ENGINE_SO=$so timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk' --output-format csv \
      -d /tmp/pmc_m_${v}_$c -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/pmc_${v}_$c.log 2>&1
    find /tmp/pmc_m_${v}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_${v}_$c.csv \;
  done
done
python3 - <<'PY'
import csv, glob, os
out = os.environ['GRAFT_REPO_ROOT'] + '/gpurun_out/r02m'
for v in ('base', 'nt'):
    tot = {}
    for c in ('FETCH_SIZE', 'WRITE_SIZE'):
        rows = list(csv.DictReader(open(f'{out}/pmc_{v}_{c}.csv')))
        vals = [float(r['Counter_Value']) for r in rows if r['Counter_Name'] == c]
        disp = len(set(r['Dispatch_Id'] for r in rows if r['Counter_Name'] == c))
        tot[c] = sum(vals) / max(disp, 1)
    print(v, 'fetch KB x2 per launch %.3g GB' % (tot['FETCH_SIZE'] * 2 * 1024 / 1e9), 'write %.3g GB' % (tot['WRITE_SIZE'] * 1024 / 1e9))
PY
