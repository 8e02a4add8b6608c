# final tree: smoke + default bench (with CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke85.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench85.json 2> gpurun_out/bench85.err || exit 1
echo "all done"
