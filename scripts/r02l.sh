#!/bin/bash
# demod A/B: cm prefetch, FIR imaginary-chain group size
set -eo pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/ab_bench.sh r02l "base pref g16 g28 prefg16" --steps 10
