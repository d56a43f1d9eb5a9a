#!/bin/bash
set -eo pipefail
bash profiles/r05/shares.sh r05 c3 8 0 3 7
GSRT_DEBUG_NO_FRONTIER=1 bash profiles/r05/shares.sh r05nf c3 8 3
bash profiles/r05/share_prof.sh c3 8 3
mv gpurun_out/r05/sp_c3_8_3_alone gpurun_out/r05/sp_c3_8_3_alone_front
GSRT_DEBUG_NO_FRONTIER=1 bash profiles/r05/share_prof.sh c3 8 3
