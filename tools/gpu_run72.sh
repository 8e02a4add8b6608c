# conv-stack weight gradients on the side stream: parity + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py tests/test_ops_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/side_tests.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo "all done"
