# the group-list depth cull evaluated only once the key buffer has overflowed (product) against on every internal child
# (libgsrt_ab.so: the previous commit)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q -k "depth_cull or pipelined or c5" --timeout 200 --timeout-method thread > gpurun_out/r06_t32.log 2>&1
rc=$?
tail -2 gpurun_out/r06_t32.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r06_t32.log | head -5; exit 1; fi
bash profiles/r06/ab.sh r06_ab32 c3 c2 c4 c5 c3:8:2
