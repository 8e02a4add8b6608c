# GPU tests, head micro-bench, rocprof kernel stats + PMC traffic passes, full bench (round-1 evidence)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/bench_head.py > gpurun_out/bench_head.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o head -- python tools/bench_head.py --iters 3 --warm 1 > gpurun_out/prof_head.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o head -- python tools/bench_head.py --iters 2 --warm 1 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o head -- python tools/bench_head.py --iters 2 --warm 1 > gpurun_out/pmc_write.log 2>&1 && \
python tools/pmc_summary.py gpurun_out/pmc_fetch/head_counter_collection.csv gpurun_out/pmc_write/head_counter_collection.csv gpurun_out/pmc_traffic.json > /dev/null && \
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 && \
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv gpurun_out/prof_head/head_kernel_trace.csv && \
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1
echo "all rc=$?"
