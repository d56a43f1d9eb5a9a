#!/bin/bash
# mesh co-tracing GPU tests, then the REF/COR render suite
set -o pipefail
O=gpurun_out/r02b_mesh
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mesh.py -x -v --timeout 120 --timeout-method thread > $O/pytest_mesh.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_render_gpu.py tests/test_bvh_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_render.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
echo ok
