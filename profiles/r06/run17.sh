# cost-driven longest-first XCD deal of a share's render units (product) against the centre-out deal (GSRT_DEBUG_DEAL=0)
set -o pipefail
AB_ENV=GSRT_DEBUG_DEAL=0 bash profiles/r06/ab.sh r06_ab17 c3:8:1 c3:8:2 c3:8:5 c3:8:7 c3:4:1 c4:8:6 c4:8:2 c5:8:5
