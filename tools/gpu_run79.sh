# qkv dW storage-sharing outputs, projection-head cast order: parity + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_head_gpu.py tests/test_postln_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t79.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo "all done"
