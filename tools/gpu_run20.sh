# forward-kernel A/B: which part bounds pairsim_fwd2 (DMA / epilogue / dS stores)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/fwd_micro.py > gpurun_out/fwd_micro.log 2>&1 || exit 1
for v in nodma noepi nostore bare epionly prio region4; do
  TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 120 python tools/fwd_micro.py >> gpurun_out/fwd_micro.log 2>&1 || exit 1
done
echo "all done"
