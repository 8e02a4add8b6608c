# round artefacts at HEAD: default bench (with the CPU baseline), kernel-trace stats of the bench,
# PMC FETCH/WRITE passes on the forward microbench (HBM traffic of the roofline kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o fwd -- python tools/fwd_micro.py --iters 2 > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o fwd -- python tools/fwd_micro.py --iters 2 > gpurun_out/pmc_write.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_fetch/fwd_counter_collection.csv gpurun_out/pmc_write/fwd_counter_collection.csv gpurun_out/pmc_traffic.json > /dev/null || exit 1
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
TRIAD_PROFILE_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 1
python tools/trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv 3 gpurun_out/bench_steady_kernels.csv > gpurun_out/trace_summary.log 2>&1
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
echo "all done"
