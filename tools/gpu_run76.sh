# GELU pass blocks per CU (2 / 3 / 4 / 8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 python tools/gelu_micro.py > gpurun_out/gelu_b2.log 2>&1 || exit 1
for v in b3 b4 b8; do
TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 100 python tools/gelu_micro.py > gpurun_out/gelu_$v.log 2>&1 || exit 1
done
echo "all done"
