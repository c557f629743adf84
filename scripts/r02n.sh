#!/bin/bash
# timing-only A/B: coarse kernel without the two bit-reversal LDS exchanges (wrong results)
set -eo pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/ab_bench.sh r02n "base skipbr" --steps 10
