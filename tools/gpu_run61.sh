# aten ops of one step by input shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/step_ops.py 90 > gpurun_out/step_ops.log 2>&1 || exit 1
echo "all done"
