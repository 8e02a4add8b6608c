# A/B of a variant build (tools/build_variants.py name="-D...") against the product library:
# parity of the variant (head tests + kernel-tour digests against the product build's), then a
# micro-benchmark alternated product / variant three times.
# usage: gpurun -- bash tools/gpu_ab_variant.sh <variant name> <tag> [micro script, default tools/fwd_micro.py]
export TMPDIR=/tmp; mkdir -p gpurun_out
v=$1; tag=$2; micro=${3:-tools/fwd_micro.py}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
export TRIAD_LIB_VARIANT=tools/variants/lib_$v.so
timeout -k 10 400 python -u -m pytest tests/test_head_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_head_tests_$v.log 2>&1 || exit 1
timeout -k 10 300 python tools/kernel_tour.py gpurun_out/${tag}_tour_$v.json > gpurun_out/${tag}_tour_$v.log 2>&1 || exit 1
unset TRIAD_LIB_VARIANT
timeout -k 10 300 python tools/kernel_tour.py gpurun_out/${tag}_tour_prod.json > gpurun_out/${tag}_tour_prod.log 2>&1 || exit 1
for r in 1 2 3; do for w in prod $v; do
  if [ $w = prod ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$w.so; fi
  timeout -k 10 180 python $micro --iters 20 --tag $w >> gpurun_out/${tag}_ab.log 2>&1 || exit 1
done; done
