#!/bin/bash
# A/B of two library builds (no parity run): bash profiles/r02c_ab_lib.sh <libA> <libB> <tag>
set -o pipefail
mkdir -p gpurun_out/$3
bash profiles/r02b_ab_all.sh $1 $2 > gpurun_out/$3/ab.log 2>&1 || exit 1
echo ok
