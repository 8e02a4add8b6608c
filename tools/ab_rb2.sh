set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V=tools/variants/lib_rb2.so
timeout -k 10 300 python tools/fwd_micro.py > gpurun_out/r03zh_fwd_a1.log 2>&1 &&
TRIAD_LIB_VARIANT=$V timeout -k 10 300 python tools/fwd_micro.py > gpurun_out/r03zh_fwd_b1.log 2>&1 &&
timeout -k 10 300 python tools/fwd_micro.py > gpurun_out/r03zh_fwd_a2.log 2>&1 &&
TRIAD_LIB_VARIANT=$V timeout -k 10 300 python tools/fwd_micro.py > gpurun_out/r03zh_fwd_b2.log 2>&1 &&
TRIAD_LIB_VARIANT=$V timeout -k 10 600 python -u -m pytest tests/test_head_gpu.py tests/test_dropin_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03zh_tests_rb2.log 2>&1
