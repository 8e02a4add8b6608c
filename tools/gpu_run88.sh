# measured dW split table: full GPU suite, then bench A/B (table off / on, twice) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/t88.log 2>&1 || exit 1
TRIAD_DW_SPLIT_TABLE=0 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench88_t0.json 2> gpurun_out/bench88_t0.err || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench88_t1.json 2> gpurun_out/bench88_t1.err || exit 1
TRIAD_DW_SPLIT_TABLE=0 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench88_t0b.json 2> gpurun_out/bench88_t0b.err || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench88_t1b.json 2> gpurun_out/bench88_t1b.err || exit 1
echo "all done"
