# the 1-GPU C5 frame with the prep streams always at the highest priority (GSRT_DEBUG_PREP_PRIORITY=1) against the rule
# (lowest above 2.5 ms of render)
set -o pipefail
AB_ENV=GSRT_DEBUG_PREP_PRIORITY=1 bash profiles/r06/ab.sh r06_ab27 c5 c5:2:0
