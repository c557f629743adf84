#!/bin/bash
# One GPU call made of named steps, each under its own time limit, output to
# gpurun_out/TAG/.  A step that fails its checks (pytest / bench exit 1-3) is
# recorded and the call goes on; a fault, abort, segfault or time limit ends it.
#   tests[=K_EXPR]     the GPU suite (or a -k subset; '+' stands for ' or ')
#   vtests=VARIANT:K   a -k subset of the GPU suite on libaero_engine_VARIANT.so
#   smoke              __graft_entry__.smoke()
#   bench[=ARGS]       bench.py (default: the headline line), ARGS comma-separated
#   mode=M             bench.py --mode M with its CPU baseline (one run)
#   ab=VARIANT:M       bench.py --mode M on libaero_engine_VARIANT.so, no CPU baseline
#   env=VAR=VALUE      export VAR=VALUE for the steps after it
#   pmcdrop            demod HBM traffic per buffer (scripts/pmc_demod_buffers.sh)
#   pmc                FETCH_SIZE / WRITE_SIZE of the headline's demod and coarse
#                      kernels (two passes) -> pmc_oqpsk10500.json
#   trace=M            rocprofv3 kernel trace of bench.py --mode M (kernel_trace_M.csv)
#   stamps[=VARIANT]   per-section cycle totals (libaero_engine_stamps.so or _VARIANT.so)
# Usage: bash scripts/gpu_steps.sh TAG STEP...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
step() {  # SECONDS OUTFILE cmd...
  local s=$1 f=$2; shift 2
  timeout -k 10 "$s" "$@" > "$OUT/$f" 2>&1
  local rc=$?
  echo "[step] rc=$rc $*" | tee -a "$OUT/$f"
  [ $rc -ge 4 ] && exit $rc
  return 0
}
for st in "$@"; do
  case $st in
    tests) step 900 pytest_gpu.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests ;;
    tests=*) k=${st#tests=}; step 900 pytest_gpu_${k//+/_}.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "${k//+/ or }" tests ;;
    vtests=*) v=${st#vtests=}; k=${v#*:}; v=${v%%:*}
      AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_$v.so step 900 pytest_gpu_${v}_${k//+/_}.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "${k//+/ or }" tests ;;
    smoke) step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step 400 bench.log python bench.py ;;
    bench=*) a=${st#bench=}; step 400 "bench_${a//[ ,=-]/_}.log" python bench.py ${a//,/ } ;;
    mode=*) m=${st#mode=}; step 400 bench_$m.log python bench.py --mode $m --cpu-runs 1 ;;
    ab=*) v=${st#ab=}; m=${v#*:}; v=${v%%:*}
      so=$R/aero-cli_amd/libaero_engine${v:+_$v}.so; [ "$v" = prod ] && so=$R/aero-cli_amd/libaero_engine.so
      AERO_ENGINE_SO=$so step 300 bench_${m}_$v${GPU_MAX_HW_QUEUES:+_q$GPU_MAX_HW_QUEUES}.log python bench.py --mode $m --no-cpu-baseline ;;
    stamps) AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_stamps.so step 300 coarse_stamps.log python -u scripts/coarse_stamps.py
      AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_stamps.so step 300 demod_stamps.log python -u scripts/demod_stamps.py ;;
    stamps=*) v=${st#stamps=}
      AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_$v.so step 300 coarse_stamps_$v.log python -u scripts/coarse_stamps.py ;;
    trace=*) m=${st#trace=}${GPU_MAX_HW_QUEUES:+_q$GPU_MAX_HW_QUEUES}
      cd /tmp; TMPDIR=/tmp step 400 trace_$m.log rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_${TAG}_$m -o tr -- python3 $R/bench.py --mode ${st#trace=} --no-cpu-baseline; cd $R
      find /tmp/tr_${TAG}_$m -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace_$m.csv \; ;;
    pmcdrop) step 900 pmcdrop.log bash scripts/pmc_demod_buffers.sh $TAG ;;
    pmc) cd /tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        TMPDIR=/tmp step 400 pmc_$c.log rocprofv3 --pmc $c --kernel-include-regex 'demod_oqpsk|coarse_kernel' --output-format csv \
          -d /tmp/pmc_${TAG}_$c -o pmc -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --h2d-steps 0
        find /tmp/pmc_${TAG}_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_$c.csv \;
      done
      cd $R
      python3 tools/pmc_json.py $OUT/pmc_FETCH_SIZE.csv $OUT/pmc_WRITE_SIZE.csv $OUT/pmc_oqpsk10500.json oqpsk10500 65536 \
        "rocprofv3 --pmc, one pass per counter, bench.py --steps 4 --warmup 1" > /dev/null ;;
    env=*) export "${st#env=}"; echo "[step] export ${st#env=}" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
