# 2x2-tile groups (GSRT_DEBUG_GROUP_TILES=2) against the default rule on the 1-GPU C2 and C4 frames and C3
set -o pipefail
AB_ENV=GSRT_DEBUG_GROUP_TILES=2 bash profiles/r06/ab.sh r06_ab22 c2 c4 c3
