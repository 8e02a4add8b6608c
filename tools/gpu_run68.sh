# weight-gradient GEMMs: ours vs tuned library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/dw_tunable.py > gpurun_out/dw_tunable.log 2>&1 || exit 1
echo "all done"
