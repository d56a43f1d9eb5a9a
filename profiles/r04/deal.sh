#!/bin/bash
# weighted root deal A/B: every rank's 8-rank C3 and C4 share at the default root weight and at GSRT_ROOT_SHARE=1
# (plain round-robin). From the repo root on the GPU box: bash profiles/r04/deal.sh <tag>
set -eo pipefail
TAG=${1:-deal}
for w in default 1; do
  if [ $w = default ]; then unset GSRT_ROOT_SHARE; else export GSRT_ROOT_SHARE=$w; fi
  echo "== root share $w"
  bash profiles/r04/shares.sh ${TAG}_$w c3 8 0 1 2 3 4 5 6 7
  bash profiles/r04/shares.sh ${TAG}_$w c4 8 0 1 2 3 4 5 6 7
done
