# forward A/B variants (setprio, scheduling region), test fix, full bench with cpu baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_head_gpu.py -q -x > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
for v in base prio r2 r8 prio_r2; do
  TRIAD_LIB_VARIANT=tools/variants/lib_$v.so timeout -k 10 300 python tools/bench_head.py --iters 10 > gpurun_out/bh_$v.log 2>&1 || break
done
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1
echo "all done"
