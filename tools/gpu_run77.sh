# head parity + HBM traffic PMC passes (FETCH_SIZE / WRITE_SIZE) for the renamed forward instantiations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o head -- python tools/bench_head.py --iters 2 --warm 1 > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o head -- python tools/bench_head.py --iters 2 --warm 1 > gpurun_out/pmc_write.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_fetch/head_counter_collection.csv gpurun_out/pmc_write/head_counter_collection.csv gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.log 2>&1 || exit 1
echo "all done"
