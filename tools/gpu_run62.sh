# HIP slab sums for LN / posconv parameter gradients: parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_postln_gpu.py tests/test_frontend_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/fe_tests.log 2>&1 || exit 1
echo "all done"
