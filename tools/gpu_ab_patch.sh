# Micro A/B of the dS max-term patch (tools/fwd_micro.py --patch) over variant builds and grid sizes,
# alternated round by round on one box.
# usage: gpurun -- bash tools/gpu_ab_patch.sh <tag> <rounds> "<nmp list>" <variant> [<variant> ...]
export TMPDIR=/tmp; mkdir -p gpurun_out
tag=$1; rounds=$2; nmps=$3; shift 3
for r in $(seq 1 $rounds); do for w in prod "$@"; do for n in $nmps; do
  if [ $w = prod ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$w.so; fi
  TRIAD_PATCH_NMP=$n timeout -k 10 120 python tools/fwd_micro.py --patch --iters 20 --tag $w >> gpurun_out/${tag}_ab.log 2>&1 || exit 1
done; done; done
