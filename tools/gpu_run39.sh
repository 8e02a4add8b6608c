# generic GEMM A/B: DMA pieces spread between MFMAs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in default gspread; do
  if [ $v = default ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$v.so; fi
  echo "== $v" >> gpurun_out/ab.log
  timeout -k 10 300 python tools/conv_micro.py >> gpurun_out/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/dw_variants.py 50944 2>&1 | grep triad >> gpurun_out/ab.log || exit 1
done
TRIAD_LIB_VARIANT=tools/variants/lib_gspread.so timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py tests/test_ops_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/tests_gspread.log 2>&1 || exit 1
echo "all done"
