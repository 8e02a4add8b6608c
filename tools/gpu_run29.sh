# stream-K tile GEMM: parity tests, microbench vs split-K
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/bwd_micro.py > gpurun_out/bwd_micro.log 2>&1 || exit 1
TRIAD_TILE_GEMM=split timeout -k 10 120 python tools/bwd_micro.py >> gpurun_out/bwd_micro.log 2>&1 || exit 1
echo "all done"
