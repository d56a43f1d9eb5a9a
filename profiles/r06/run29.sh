# three group-list segments (libgsrt_ab.so, -DGSRT_GROUP_SEGMENTS=3) against two (product)
set -o pipefail
bash profiles/r06/ab.sh r06_ab29 c5 c5:8:5 c5:8:1 c5:4:1
