# relaxed dS-store vmcnt in the forward; 4-slot ring tile GEMM vs the 2-stage form; head parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_head_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/fwd_micro.py > gpurun_out/fwd_micro.log 2>&1 || exit 1
timeout -k 10 120 python tools/bwd_micro.py > gpurun_out/bwd_micro.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_tgold.so timeout -k 10 120 python tools/bwd_micro.py >> gpurun_out/bwd_micro.log 2>&1 || exit 1
echo "all done"
