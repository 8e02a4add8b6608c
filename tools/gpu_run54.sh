# steady-state kernel trace of the current step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TRIAD_PROFILE_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 1
python tools/trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv 3 gpurun_out/bench_steady_kernels.csv > gpurun_out/trace_summary.log 2>&1
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
echo "all done"
