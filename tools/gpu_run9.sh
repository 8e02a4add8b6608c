# v2 (pipelined) forward: parity under TRIAD_FWD_V2=1, head timing v1 vs v2, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 env TRIAD_FWD_V2=1 python -m pytest tests/test_head_gpu.py tests/test_retrieval_gpu.py tests/test_dist_gpu.py -q -x > gpurun_out/gpu_tests_v2.log 2>&1
echo "v2 tests rc=$?" >> gpurun_out/gpu_tests_v2.log
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -q -x > gpurun_out/gpu_tests_ops.log 2>&1
echo "ops tests rc=$?" >> gpurun_out/gpu_tests_ops.log
timeout -k 10 300 python tools/bench_head.py > gpurun_out/bench_head_v1.log 2>&1 && \
timeout -k 10 300 env TRIAD_FWD_V2=1 python tools/bench_head.py > gpurun_out/bench_head_v2.log 2>&1 && \
TRIAD_FWD_V2=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head_v2 -o head -- python tools/bench_head.py --iters 3 --warm 1 > gpurun_out/prof_head_v2.log 2>&1 && \
rm -f gpurun_out/prof_head_v2/head_kernel_trace.csv
echo "all rc=$?"
