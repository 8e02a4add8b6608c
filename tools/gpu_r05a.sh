export TMPDIR=/tmp; mkdir -p gpurun_out
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
unset TRIAD_LIB_VARIANT
timeout -k 10 300 python tools/kernel_tour.py gpurun_out/r05a_tour_prod.json > gpurun_out/r05a_tour_prod.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_head_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05a_head_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_projhead_gpu.py tests/test_ops_gpu.py -m gpu -q -k "projection or bias_grad or colsum or strided or similarity" --timeout 300 --timeout-method thread > gpurun_out/r05a_proj_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05a_projk -o run -- python3 tools/projhead_kernels.py --iters 10 > gpurun_out/r05a_projk.log 2>&1 || exit 1
for r in 1 2; do for v in 0 1 2 3 4; do
  if [ $v = 0 ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_dsst$v.so; fi
  timeout -k 10 120 python tools/fwd_micro.py --iters 30 --tag dsst$v >> gpurun_out/r05a_fwd_store_ab.log 2>&1 || exit 1
done; done
unset TRIAD_LIB_VARIANT
TRIAD_LIB_VARIANT=tools/variants/lib_ldscheck.so timeout -k 10 300 python tools/kernel_tour.py gpurun_out/r05a_tour_ldscheck.json > gpurun_out/r05a_tour_ldscheck.log 2> gpurun_out/r05a_tour_ldscheck.err; echo "ldscheck tour rc=$?" >> gpurun_out/r05a_tour_ldscheck.err
