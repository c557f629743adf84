#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/ab_bench.sh r03r "base corunp corunp8" --steps 20 --warmup 5
