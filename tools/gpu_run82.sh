# N=2 rehearsal of bench.py's distributed path on the one-GPU box (gloo, both ranks on cuda:0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TRIAD_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 \
  > gpurun_out/bench82_n2.json 2> gpurun_out/bench82_n2.err || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 32 --no-cpu-baseline \
  > gpurun_out/bench82_n1.json 2> gpurun_out/bench82_n1.err || exit 1
echo "all done"
