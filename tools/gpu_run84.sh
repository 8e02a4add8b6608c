# host enqueue time per step vs wall time per step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/host_enqueue.py > gpurun_out/host84.json 2> gpurun_out/host84.err || exit 1
echo "all done"
