# the group-list traversal without its depth cull (libgsrt_xnodc.so) and without the new-tail merge (libgsrt_xnomg.so)
# against the product, on the configs whose lists rarely overflow (C2, C3, C4) and on C5
set -o pipefail
cp 3dgs-raytrace_amd/gsrt/libgsrt_xnodc.so 3dgs-raytrace_amd/gsrt/libgsrt_ab.so && \
bash profiles/r06/ab.sh r06_ab30_nodc c2 c3 c4 c5 && \
cp 3dgs-raytrace_amd/gsrt/libgsrt_xnomg.so 3dgs-raytrace_amd/gsrt/libgsrt_ab.so && \
bash profiles/r06/ab.sh r06_ab30_nomg c2 c3 c4 c5
