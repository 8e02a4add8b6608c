# posconv forward with LDS-staged weights: parity + micro
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py -k pos -x -q --timeout 250 --timeout-method thread > gpurun_out/fe_tests.log 2>&1 || exit 1
timeout -k 10 100 python tools/posconv_micro.py > gpurun_out/pc_lds.log 2>&1 || exit 1
echo "all done"
