# host-sync removal (pinned H2D, cached index tensors, SpecAugment without boolean assignment, no-pad text mask):
# all GPU tests, bench, steady profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
TRIAD_PROFILE_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 && \
python tools/trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv 3 gpurun_out/bench_steady_kernels.csv > gpurun_out/trace_summary.log 2>&1
python - <<'PY' > gpurun_out/gaps.txt 2>&1
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_bench/bench_kernel_trace.csv")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows)
gaps = []
for a, b in zip(ev, ev[1:]):
    g = b[0] - a[1]
    if g > 200000:
        gaps.append((g / 1e6, a[2], b[2]))
gaps.sort(reverse=True)
for g in gaps[:40]:
    print("%.2f ms  after %s  before %s" % g)
print("total gaps > 0.2 ms:", sum(g[0] for g in gaps))
PY
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
echo "all done"
