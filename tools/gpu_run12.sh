# asm-hidden LDS-DMA forward, bf16 model weights: parity, head timing, SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/bench_head.py > gpurun_out/bench_head.log 2>&1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
timeout -k 10 300 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/sq1 -o head -- python tools/bench_head.py --iters 1 --warm 1 > gpurun_out/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/sq2 -o head -- python tools/bench_head.py --iters 1 --warm 1 > gpurun_out/sq2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o head -- python tools/bench_head.py --iters 3 --warm 1 > gpurun_out/prof_head.log 2>&1
rm -f gpurun_out/prof_head/head_kernel_trace.csv
echo "all done"
TRIAD_PROFILE_MARK=1 timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 && \
python tools/trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv 3 gpurun_out/bench_steady_kernels.csv > gpurun_out/trace_summary.log 2>&1
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
echo "bench profile done"
