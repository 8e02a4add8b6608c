# A/B of the forward: DMA pieces spread between MFMAs, s_setprio, LDS read depth (scalar epilogue pairs now default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
for v in default fwdspread fwdprio fwdspreadprio fwdpf3 default fwdspread; do
  if [ $v = default ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$v.so; fi
  timeout -k 10 120 python tools/fwd_micro.py >> gpurun_out/ab.log 2>&1 || exit 1
done
unset TRIAD_LIB_VARIANT
timeout -k 10 120 python tools/bwd_micro.py >> gpurun_out/ab.log 2>&1 || exit 1
TRIAD_LIB_VARIANT=tools/variants/lib_fwdspread.so timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/head_tests_fwdspread.log 2>&1 || exit 1
echo "all done"
