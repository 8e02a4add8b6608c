# A/B of the direct-B tile GEMM stage shapes (round 3; the variants were built with
# tools/build_variants.py from -DTRIAD_DB_KS / -DTRIAD_DB_D knobs since replaced by per-GEMM template
# parameters in bwd_gemm.hip -- kept as the record of how profiles/r03_tile_gemm_db_ab.log was made):
# default (1 k tile per stage, 3 stages ahead) vs 2 tiles per stage (1 / 2 stages ahead) and 1 x 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in default ks2d1 ks2d2 ks1d4; do
    if [ $v = default ]; then unset TRIAD_LIB_VARIANT; else export TRIAD_LIB_VARIANT=tools/variants/lib_$v.so; fi
    timeout -k 10 300 python tools/bwd_micro.py --forms 0,9 > gpurun_out/r03d_db_${v}_$r.log 2>&1 || exit 1
  done
done
