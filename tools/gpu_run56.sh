# posconv forward B-prefetch distance (2 / 4 / 8) + parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py -k pos -x -q --timeout 250 --timeout-method thread > gpurun_out/fe_tests.log 2>&1 || exit 1
timeout -k 10 100 python tools/posconv_micro.py > gpurun_out/pc_pd4.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_pd2.so timeout -k 10 100 python tools/posconv_micro.py > gpurun_out/pc_pd2.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_pd8.so timeout -k 10 100 python tools/posconv_micro.py > gpurun_out/pc_pd8.log 2>&1 || exit 1
echo "all done"
