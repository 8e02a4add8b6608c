# HuBERT execution tweaks (channels-last convs, no waveform grad): tests, steady bench profile,
# PMC FETCH/WRITE passes on the head (traffic for the roofline line)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o head -- python tools/bench_head.py --iters 2 --warm 1 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o head -- python tools/bench_head.py --iters 2 --warm 1 > gpurun_out/pmc_write.log 2>&1 && \
python tools/pmc_summary.py gpurun_out/pmc_fetch/head_counter_collection.csv gpurun_out/pmc_write/head_counter_collection.csv gpurun_out/pmc_traffic.json > /dev/null
TRIAD_PROFILE_MARK=1 timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 && \
python tools/trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv 3 gpurun_out/bench_steady_kernels.csv > gpurun_out/trace_summary.log 2>&1
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
echo "all done"
