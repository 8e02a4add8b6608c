# c5-size head parity; per-backbone kernel attribution
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || exit 1
for m in vit hubert distilbert; do
  timeout -k 10 300 python tools/backbone_profile.py $m > gpurun_out/bb_$m.log 2>&1 || exit 1
done
echo "all done"
