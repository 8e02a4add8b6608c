# A/B: scalar epilogue pairs in the forward; DMA pieces spread between MFMAs in the tile GEMM
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in default fwdscalar tgspread default; do
  if [ $v = default ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$v.so; fi
  timeout -k 10 120 python tools/fwd_micro.py >> gpurun_out/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bwd_micro.py >> gpurun_out/ab.log 2>&1 || exit 1
done
for v in fwdscalar tgspread; do
  TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/head_tests_$v.log 2>&1 || exit 1
done
echo "all done"
