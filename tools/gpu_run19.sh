# u-domain forward epilogue: head parity tests, all GPU tests, head microbench + kernel stats, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o head -- python tools/bench_head.py --iters 3 --warm 1 > gpurun_out/prof_head.log 2>&1 || exit 1
rm -f gpurun_out/prof_head/head_kernel_trace.csv
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo "all done"
