# attention kernels: SQ counters (issue / wait breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-include-regex attn --output-format csv -d gpurun_out/pmc_attn -o attn -- python tools/attn_micro.py > gpurun_out/pmc_attn.log 2>&1 || exit 1
echo "all done"
