# forward-kernel A/B: nt stores, LDS read depth, 2-slot ring, 4-wave workgroups (2 per CU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/fwd_micro.py > gpurun_out/fwd_micro.log 2>&1 || exit 1
for v in nt pf3 nb2 w4 w4nt; do
  TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 120 python tools/fwd_micro.py >> gpurun_out/fwd_micro.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/fwd_micro.py >> gpurun_out/fwd_micro.log 2>&1 || exit 1
echo "all done"
