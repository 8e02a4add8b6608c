# modality streams: single- vs multi-stream step parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k modality_streams -x -q --timeout 250 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || exit 1
echo "all done"
