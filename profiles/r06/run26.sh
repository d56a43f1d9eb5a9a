# prep streams at the lowest priority (GSRT_DEBUG_PREP_PRIORITY=0) against the rule (highest below 2 ms of render), now
# that three slots give the chain two renders of lead
set -o pipefail
AB_ENV=GSRT_DEBUG_PREP_PRIORITY=0 bash profiles/r06/ab.sh r06_ab26 c5:8:5 c5:8:1 c5:4:1 c3:4:1 c3 c3:2:1
