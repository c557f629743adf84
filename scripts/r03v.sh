#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/ab_bench.sh r03v "base nobperm" --steps 10 --warmup 3
