# round artifacts: full GPU suite + smoke + default bench (with CPU baseline) + steady trace + rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
TRIAD_PROFILE_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 1
python tools/trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv 3 gpurun_out/bench_steady_kernels.csv > gpurun_out/trace_summary.log 2>&1
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
echo "all done"
