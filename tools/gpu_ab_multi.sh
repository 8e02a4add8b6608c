# Micro A/B of several variant builds (tools/build_variants.py) against the product library,
# alternated round by round on one box; timing only (parity of a chosen variant: gpu_ab_variant.sh).
# usage: gpurun -- bash tools/gpu_ab_multi.sh <tag> <rounds> <variant> [<variant> ...]
# MICRO="tools/bwd_micro.py --forms 16 --ct 1656,1656" selects another micro (default: the forward's)
export TMPDIR=/tmp; mkdir -p gpurun_out
tag=$1; rounds=$2; shift 2
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
for r in $(seq 1 $rounds); do for w in prod "$@"; do
  if [ $w = prod ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$w.so; fi
  timeout -k 10 180 python ${MICRO:-tools/fwd_micro.py} --iters 20 --tag $w >> gpurun_out/${tag}_ab.log 2>&1 || exit 1
done; done
