# A/B of the dS load cache policy in the direct-B backward tile GEMMs (TRIAD_DS_LOAD_POL variants
# built by tools/build_variants.py) + the similarity-map tests and rocprof evidence.
export TMPDIR=/tmp; mkdir -p gpurun_out
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
unset TRIAD_LIB_VARIANT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_dropin_gpu.py -m gpu -q -k "similarity or simmat" --timeout 120 --timeout-method thread > gpurun_out/r05m_simmap_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05m_simmap -o run -- python3 tools/simmap_trace.py --calls 5 > gpurun_out/r05m_simmap.log 2>&1 || exit 1
for r in 1 2; do for v in 0 1 2 3; do
  if [ $v = 0 ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_dsld$v.so; fi
  timeout -k 10 180 python tools/bwd_micro.py --iters 20 --forms 16 --tag dsld$v >> gpurun_out/r05m_bwd_dsload_ab.log 2>&1 || exit 1
done; done
