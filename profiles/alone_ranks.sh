set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/alone
for r in 0 4 2 6; do
  GSRT_DEBUG_RANK_OF=8:$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/alone/r$r -o run -- python3 profiles/alone.py c3 40 > gpurun_out/alone/r$r.log 2>&1
done
echo ok
