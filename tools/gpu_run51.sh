# four-wave GEMM: DMA piece spacing (GW_EVERY 1 / 2 / 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_forms.py > gpurun_out/gf_e2.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_e1.so timeout -k 10 200 python tools/gemm_forms.py > gpurun_out/gf_e1.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_e4.so timeout -k 10 200 python tools/gemm_forms.py > gpurun_out/gf_e4.log 2>&1 || exit 1
echo done
