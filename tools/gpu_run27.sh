# forward A/B bounds (no stores / no epilogue / no DMA / bare chain) + backward tile GEMM microbench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/fwd_micro.py > gpurun_out/fwd_micro.log 2>&1 || exit 1
for v in nostore noepi nodma bare; do
  TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 120 python tools/fwd_micro.py >> gpurun_out/fwd_micro.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/bwd_micro.py > gpurun_out/bwd_micro.log 2>&1 || exit 1
echo "all done"
