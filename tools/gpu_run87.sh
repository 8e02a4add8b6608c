# dW split-K factor sweep incl. non-power-of-two splits (HuBERT 50,944 and DistilBERT 8,192 tokens)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TRIAD_DW_SPLITS=4,5,6,7,8,9,10,12 timeout -k 10 300 python tools/dw_variants.py 50944 > gpurun_out/dw87_50944.log 2>&1 || exit 1
TRIAD_DW_SPLITS=2,3,4,5,6,7,8 timeout -k 10 300 python tools/dw_variants.py 8192 > gpurun_out/dw87_8192.log 2>&1 || exit 1
echo "all done"
