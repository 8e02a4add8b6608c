# final HEAD: smoke, default bench (CPU baseline), rocprofv3 kernel stats of a 3-step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke90.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench90.json 2> gpurun_out/bench90.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof90 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof90_bench.json 2> gpurun_out/prof90.err || exit 1
find gpurun_out/prof90 -name "*kernel_stats.csv" > gpurun_out/prof90_files.txt
echo "all done"
