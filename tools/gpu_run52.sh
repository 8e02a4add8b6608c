# four-wave ring GEMM form: parity + form comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_head_gpu.py -k gemm_layouts -x -q --timeout 100 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/gemm_forms.py > gpurun_out/gemm_forms.log 2>&1 || exit 1
echo done
