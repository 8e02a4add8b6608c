set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/bench_head.py > gpurun_out/bench_head.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o head -- python tools/bench_head.py --iters 3 --warm 1 > gpurun_out/prof_head.log 2>&1
