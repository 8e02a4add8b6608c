# backbone attention kernels: parity tests + microbench vs torch SDPA
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_micro.py > gpurun_out/attn_micro.log 2>&1 || exit 1
echo "all done"
