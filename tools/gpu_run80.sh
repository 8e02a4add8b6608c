# side-stream join per graph task: bit-identity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_frontend_gpu.py -k "side_stream or modality" -x -q --timeout 250 --timeout-method thread > gpurun_out/t80.log 2>&1 || exit 1
echo "all done"
