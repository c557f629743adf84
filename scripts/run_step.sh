#!/bin/bash
# One GPU step under its own time limit, output to gpurun_out/<file>.
# Usage: bash scripts/run_step.sh SECONDS OUTFILE cmd args...
# Exit status: 0 when the step passed or only failed its checks (pytest /
# bench exit 1-3: results to read), the step's own status after a fault,
# abort, segfault or time limit (then the calling script must stop).
S=$1; OUT=$2; shift 2
mkdir -p "$(dirname "$OUT")"
timeout -k 10 "$S" "$@" > "$OUT" 2>&1
rc=$?
echo "[run_step] rc=$rc $*" >> "$OUT"
tail -2 "$OUT"
if [ $rc -ge 4 ]; then exit $rc; fi
exit 0
