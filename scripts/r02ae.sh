#!/bin/bash
# price each bit-exact libm function of the OQPSK demod: device ocml for all / atan2 / hypot / the event step's tanh+sincos
set -eo pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/ab_bench.sh r02ae "base ocml oatan ohyp oev" --steps 10
