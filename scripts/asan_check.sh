#!/bin/bash
# The CPU tests against AddressSanitizer + UndefinedBehaviorSanitizer builds
# of every host-compiled source they load (aero-cli_amd/build.py --asan):
# oracle, synthetic transmitter, the device libm's host build, the engine's
# host C++ (acars_host, tables_host), the drop-in host binaries.  Python
# itself is not instrumented: the runtime is preloaded, leaks are not
# reported (the interpreter's own would drown them), any error aborts.
# Usage: bash scripts/asan_check.sh [pytest args]   (CPU only, this container)
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
python3 aero-cli_amd/build.py --asan -j 8 > /dev/null
A=$R/aero-cli_amd/build/asan
export AERO_ORACLE_SO=$A/liboracle.so AERO_SYNTH_SO=$A/libaero_synth.so AERO_MATHHOST_SO=$A/libaero_mathhost.so \
       AERO_HOSTCHECK_SO=$A/libaero_hostcheck.so AERO_HOST_BIN=$A/bin
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
exec python3 -m pytest -q -m "not gpu" -p no:cacheprovider \
  tests/test_oracle_kat.py tests/test_oracle_roundtrip.py tests/test_oracle_msk.py tests/test_oracle_burst.py \
  tests/test_oracle_burst_msk.py tests/test_oracle_pub.py tests/test_golden.py tests/test_viterbi_oracle.py \
  tests/test_math_host.py tests/test_hostcheck.py tests/test_host_output.py "$@"
