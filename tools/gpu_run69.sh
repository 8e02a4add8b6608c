# attention dropout mask kernel restructure: parity + HuBERT profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_postln_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/backbone_profile.py hubert > gpurun_out/bb_hubert.log 2>&1 || exit 1
echo "all done"
