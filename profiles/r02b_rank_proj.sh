set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_render_gpu.py tests/test_configs_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_p.log 2>&1; tail -1 gpurun_out/pt_p.log
for cfg in c3 c4; do for r in 1 2; do for lib in libgsrt_xbase libgsrt_xdeal; do
GSRT_LIB_PATH=3dgs-raytrace_amd/gsrt/$lib.so GSRT_DEBUG_RANK_OF=8 timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/rk_${cfg}_${lib}_$r.log 2>&1 || exit 1
echo "$cfg $lib r$r: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frame_ms_events": [0-9.]*' gpurun_out/rk_${cfg}_${lib}_$r.log | tr "\n" " ")"
done; done; done
