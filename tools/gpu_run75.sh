# audio stream priority A/B (0 vs -1) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TRIAD_AUDIO_STREAM_PRIORITY=0 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_p0.json 2> gpurun_out/bench_p0.err || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
TRIAD_AUDIO_STREAM_PRIORITY=0 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_p0b.json 2> gpurun_out/bench_p0b.err || exit 1
echo "all done"
