# TriadLinear (HIP split-K weight gradients in HuBERT / DistilBERT): parity, DistilBERT-size dW A/B, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ops_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/dw_variants.py 8192 > gpurun_out/dw8192.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo "all done"
