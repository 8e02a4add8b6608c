# GEMM forms: 128x128 / 256x128 ring / 256x256 four-wave on conv, dW and linear shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_forms.py > gpurun_out/gemm_forms.log 2>&1 || exit 1
echo done
