# One parameterised GPU-box runner (replaces the round-1 one-off tools/gpu_run*.sh scripts).
#
# usage (from this container):
#   gpurun --timeout 1200 -- bash tools/gpu.sh <tag> <step> [<step> ...]
# steps (run in order; the first failing / timed-out step ends the call, nothing later touches the GPU):
#   tests            full `pytest -m gpu` suite                      -> gpurun_out/<tag>_tests.log
#   tests:<expr>     `pytest -m gpu -k <expr>`                        -> gpurun_out/<tag>_tests.log
#   testsnx[:<expr>] the same without -x; test failures do not end the call
#   smoke            __graft_entry__.smoke()                          -> gpurun_out/<tag>_smoke.log
#   bench            default bench.py line (with the CPU baseline)    -> gpurun_out/<tag>_bench.json
#   benchq           bench.py --no-cpu-baseline                       -> gpurun_out/<tag>_benchq.json
#   benchenv:A=1,B=2 benchq with extra env for this step             -> gpurun_out/<tag>_benchenv<N>.json
#   prof             rocprofv3 --kernel-trace --stats of a 3-step bench -> gpurun_out/<tag>_prof/
#   pmc:<name>:<counters>  one rocprofv3 --pmc pass (counters comma-separated) of a 3-step bench
#   py:<script args>       python <script> (tools/ micro-benchmarks)    -> gpurun_out/<tag>_py<N>.log
#   envpy:A=1,B=2:<script args>  the same with extra environment for this step
#   profpy:<script args>   the same under rocprofv3 --kernel-trace --stats -> gpurun_out/<tag>_profpy<N>/
#   envprofpy:A=1,B=2:<script args>  profpy with extra environment for this step
#   pmcpy:<name>:<counters>:<script args>  one rocprofv3 --pmc pass over a python script
#   envpmcpy:A=1:<name>:<counters>:<script args>  the same with extra environment for this step
# environment: extra env for every step may be given as STEP_ENV="A=1 B=2" (exported first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; shift
[ -n "$STEP_ENV" ] && export $STEP_ENV
# heartbeat: long single steps (model builds, large parity tests) print nothing for minutes;
# every step still runs under its own `timeout`
( while sleep 50; do echo "[gpu.sh] $(date +%T) running"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
n=0
for step in "$@"; do
  n=$((n + 1))
  echo "[gpu.sh] $(date +%T) step $n: $step"
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "gpurun_out/${tag}_tests.log" 2>&1 ;;
    tests:*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread \
        -k "${step#tests:}" > "gpurun_out/${tag}_tests.log" 2>&1 ;;
    testsnx|testsnx:*)
      # every test runs (no -x); ordinary test failures (pytest rc 1) do not end the call
      expr=${step#testsnx}; expr=${expr#:}
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
        ${expr:+-k "$expr"} > "gpurun_out/${tag}_tests.log" 2>&1
      rc=$?; [ $rc -eq 1 ] && { echo "[gpu.sh] test failures (see log); continuing"; rc=0; }
      [ $rc -ne 0 ] && { echo "[gpu.sh] step $n ($step) failed rc=$rc"; exit $rc; }
      continue ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${tag}_smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 900 python bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err" ;;
    benchq)
      timeout -k 10 600 python bench.py --no-cpu-baseline > "gpurun_out/${tag}_benchq.json" \
        2> "gpurun_out/${tag}_benchq.err" ;;
    benchenv:*)
      # benchq with extra environment for this step only: benchenv:A=1,B=2
      ev=${step#benchenv:}
      ( export ${ev//,/ }; timeout -k 10 600 python bench.py --no-cpu-baseline ) > "gpurun_out/${tag}_benchenv${n}.json" \
        2> "gpurun_out/${tag}_benchenv${n}.err" ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${tag}_prof" -o bench \
        -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --separate-steps 0 \
        --single-stream-steps 0 --no-stream-check > "gpurun_out/${tag}_prof.log" 2>&1 ;;
    pmc:*)
      rest=${step#pmc:}; name=${rest%%:*}; ctr=${rest#*:}
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "gpurun_out/${tag}_pmc_${name}" -o run \
        -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --separate-steps 0 \
        --single-stream-steps 0 --no-stream-check > "gpurun_out/${tag}_pmc_${name}.log" 2>&1 ;;
    profpy:*)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${tag}_profpy${n}" -o run \
        -- python3 ${step#profpy:} > "gpurun_out/${tag}_profpy${n}.log" 2>&1 ;;
    envprofpy:*)
      # envprofpy:A=1,B=2:<script args>  profpy with extra environment for this step only
      rest=${step#envprofpy:}; ev=${rest%%:*}; script=${rest#*:}
      ( export ${ev//,/ }; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "gpurun_out/${tag}_profpy${n}" -o run -- python3 $script ) > "gpurun_out/${tag}_profpy${n}.log" 2>&1 ;;
    pmcpy:*)
      rest=${step#pmcpy:}; name=${rest%%:*}; rest=${rest#*:}; ctr=${rest%%:*}; script=${rest#*:}
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "gpurun_out/${tag}_pmcpy_${name}" -o run \
        -- python3 $script > "gpurun_out/${tag}_pmcpy_${name}.log" 2>&1 ;;
    envpmcpy:*)
      # envpmcpy:A=1,B=2:<name>:<counters>:<script args>  pmcpy with extra environment for this step only
      rest=${step#envpmcpy:}; ev=${rest%%:*}; rest=${rest#*:}; name=${rest%%:*}; rest=${rest#*:}
      ctr=${rest%%:*}; script=${rest#*:}
      ( export ${ev//,/ }; timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv \
        -d "gpurun_out/${tag}_pmcpy_${name}" -o run -- python3 $script ) > "gpurun_out/${tag}_pmcpy_${name}.log" 2>&1 ;;
    py:*)
      timeout -k 10 600 python ${step#py:} > "gpurun_out/${tag}_py${n}.log" 2>&1 ;;
    envpy:*)
      # envpy:A=1,B=2:<script args>  python with extra environment for this step only
      rest=${step#envpy:}; ev=${rest%%:*}; script=${rest#*:}
      ( export ${ev//,/ }; timeout -k 10 600 python $script ) > "gpurun_out/${tag}_py${n}.log" 2>&1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] step $n ($step) failed rc=$rc"; exit $rc
  fi
done
echo "[gpu.sh] all done"
