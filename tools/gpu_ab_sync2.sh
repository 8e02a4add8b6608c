# A/B of one ring barrier per two key tiles in the pair forward (TRIAD_FWD_SYNC2 variant built by
# tools/build_variants.py): parity of the variant (head tests + kernel-tour digests against the
# product build), then the forward micro alternated product / variant.
export TMPDIR=/tmp; mkdir -p gpurun_out
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
export TRIAD_LIB_VARIANT=tools/variants/lib_sync2.so
timeout -k 10 400 python -u -m pytest tests/test_head_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05s_head_tests_sync2.log 2>&1 || exit 1
timeout -k 10 300 python tools/kernel_tour.py gpurun_out/r05s_tour_sync2.json > gpurun_out/r05s_tour_sync2.log 2>&1 || exit 1
unset TRIAD_LIB_VARIANT
timeout -k 10 300 python tools/kernel_tour.py gpurun_out/r05s_tour_prod.json > gpurun_out/r05s_tour_prod.log 2>&1 || exit 1
for r in 1 2 3; do for v in prod sync2; do
  if [ $v = prod ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$v.so; fi
  timeout -k 10 180 python tools/fwd_micro.py --iters 20 --tag $v >> gpurun_out/r05s_fwd_sync2_ab.log 2>&1 || exit 1
done; done
