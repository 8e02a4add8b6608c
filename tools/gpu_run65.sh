# TunableOp probe on the c3 step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tunable_probe.py 5 80 > gpurun_out/tunable.log 2>&1 || exit 1
echo "all done"
