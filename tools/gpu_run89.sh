# dW split table A/B after a discarded warm-up run, 10 timed steps each, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench89_warm.json 2> gpurun_out/bench89_warm.err || exit 1
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench89_t1_$i.json 2> gpurun_out/bench89_t1_$i.err || exit 1
  TRIAD_DW_SPLIT_TABLE=0 timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench89_t0_$i.json 2> gpurun_out/bench89_t0_$i.err || exit 1
done
echo "all done"
