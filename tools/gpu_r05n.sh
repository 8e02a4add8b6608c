export TMPDIR=/tmp; mkdir -p gpurun_out
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_dropin_gpu.py tests/test_head_gpu.py -m gpu -q -k "similarity or simmat or tile_gemm or pair or head" --timeout 120 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05n_simmap -o run -- python3 tools/simmap_trace.py --calls 5 > gpurun_out/r05n_simmap.log 2>&1 || exit 1
timeout -k 10 300 python tools/kernel_tour.py gpurun_out/r05n_tour.json > gpurun_out/r05n_tour.log 2>&1 || exit 1
