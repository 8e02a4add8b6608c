# bias-gradient column sums on the side stream: full GPU suite, then bench A/B on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/t83.log 2>&1 || exit 1
TRIAD_SIDE_STREAM_DB=0 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench83_db0.json 2> gpurun_out/bench83_db0.err || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench83_db1.json 2> gpurun_out/bench83_db1.err || exit 1
TRIAD_SIDE_STREAM_DB=0 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench83_db0b.json 2> gpurun_out/bench83_db0b.err || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench83_db1b.json 2> gpurun_out/bench83_db1b.err || exit 1
echo "all done"
