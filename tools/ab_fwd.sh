# A/B of pair-forward variants (tools/build_variants.py): default vs $1 (tools/variants/lib_$1.so), alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do
  unset TRIAD_LIB_VARIANT
  timeout -k 10 300 python tools/fwd_micro.py > gpurun_out/r03_fwdab_default_$r.log 2>&1 || exit 1
  TRIAD_LIB_VARIANT=tools/variants/lib_$1.so timeout -k 10 300 python tools/fwd_micro.py > gpurun_out/r03_fwdab_$1_$r.log 2>&1 || exit 1
done
