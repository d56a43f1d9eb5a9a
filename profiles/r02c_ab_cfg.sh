#!/bin/bash
# Parity (bvh/config/render GPU tests) on the product library, then an A/B of a baseline library against it on the
# given configs (two interleaved rounds) and a kernel trace of the product on the first config.
#   bash profiles/r02c_ab_cfg.sh <baseline lib> <tag> <config>...
set -o pipefail
A=$1; T=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bvh_gpu.py tests/test_configs_gpu.py tests/test_render_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for c in "$@"; do for r in 1 2; do for lib in $A libgsrt; do
  GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so timeout -k 10 150 python bench.py --config $c --no-cpu-baseline > $O/${c}_${lib}_$r.log 2>&1 || exit 2
  echo "$c $lib r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/${c}_${lib}_$r.log | tr "\n" " ")" >> $O/ab.log
done; done; done
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --config $1 --steps 20 --warmup 5 --no-cpu-baseline --no-stats > $O/trace.log 2>&1 || exit 3
echo ok
