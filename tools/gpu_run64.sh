# attention: per-wave loads before the LDS staging (A/B vs previous build) + parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_old.so timeout -k 10 200 python tools/attn_micro.py > gpurun_out/attn_old.log 2>&1 || exit 1
timeout -k 10 200 python tools/attn_micro.py > gpurun_out/attn_new.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_old.so timeout -k 10 200 python tools/attn_micro.py > gpurun_out/attn_old2.log 2>&1 || exit 1
echo "all done"
