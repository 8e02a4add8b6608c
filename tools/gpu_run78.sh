# split-K dW: LDS-DMA vs register staging (128 x 128 form)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 python tools/dw_forms.py > gpurun_out/dw_dma.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_rs.so timeout -k 10 100 python tools/dw_forms.py > gpurun_out/dw_rs.log 2>&1 || exit 1
timeout -k 10 100 python tools/dw_forms.py > gpurun_out/dw_dma2.log 2>&1 || exit 1
echo "all done"
