#!/bin/bash
# runs profiles/probes/lds_bcast_probe (built here: hipcc -O3 --offload-arch=gfx950) with timing and one PMC pass
set -o pipefail
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
timeout -k 10 60 profiles/probes/lds_bcast_probe > gpurun_out/probe/time.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/probe/pmc -o run -- profiles/probes/lds_bcast_probe > gpurun_out/probe/pmc.log 2>&1 || exit 2
echo ok
