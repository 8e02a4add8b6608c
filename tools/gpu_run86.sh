# forward A/B: non-temporal dS stores, 4-wave workgroups, vs default (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/fwd_micro.py --iters 30 > gpurun_out/fwd86.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_nt.so timeout -k 10 200 python tools/fwd_micro.py --iters 30 >> gpurun_out/fwd86.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_w4.so timeout -k 10 200 python tools/fwd_micro.py --iters 30 >> gpurun_out/fwd86.log 2>&1 || exit 1
timeout -k 10 200 python tools/fwd_micro.py --iters 30 >> gpurun_out/fwd86.log 2>&1 || exit 1
echo "all done"
