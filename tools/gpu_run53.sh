# four-wave GEMM bounds: no fragment reads / no DMA / neither
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_forms.py > gpurun_out/gf_base.log 2>&1 || exit 1
for v in nolds nodma both; do
TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 200 python tools/gemm_forms.py > gpurun_out/gf_$v.log 2>&1 || exit 1
done
echo done
