# rebuilt tree (fresh container): full GPU suite, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/t81.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke81.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench81.json 2> gpurun_out/bench81.err || exit 1
echo "all done"
