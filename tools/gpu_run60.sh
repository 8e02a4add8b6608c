# fused q/k/v projection for HuBERT self-attention: parity + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_postln_gpu.py tests/test_attention_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo "all done"
