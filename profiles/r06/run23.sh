# two-stream scheme with three slots (GSRT_DEBUG_SLOT_STREAMS=0) against the adaptive choice (product: slot streams
# for short frames, two slots)
set -o pipefail
AB_ENV=GSRT_DEBUG_SLOT_STREAMS=0 bash profiles/r06/ab.sh r06_ab23 c4 c2 c3:8:2 c4:8:6 c3:8:0
