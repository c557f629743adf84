#!/bin/bash
# A/B: Viterbi grid capped at k x CUs beside the demod (g<k>), demod wave priority (p)
set -eo pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/ab_bench.sh r02v "base g1 g1p g2p g4p" --steps 10
