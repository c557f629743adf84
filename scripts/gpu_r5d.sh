#!/bin/bash
# round 5: selected GPU tests, smoke, the default bench line, then the coarse
# and demod section stamps.  Usage: bash scripts/gpu_r5d.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_check.sh $TAG "math or parity or msk or burst or handoff or events" || exit $?
bash $R/scripts/gpu_stamps.sh $TAG
