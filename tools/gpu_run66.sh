# committed TunableOp results: bench with and without (same box), trainer tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TRIAD_TUNABLEOP=0 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_off.json 2> gpurun_out/bench_off.err || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k trainer -x -q --timeout 250 --timeout-method thread > gpurun_out/trainer_tests.log 2>&1 || exit 1
echo "all done"
