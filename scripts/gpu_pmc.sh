#!/bin/bash
# PMC counters of the flagship step (two passes, each within the per-block counter limits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc1" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph > "$R/gpurun_out/pmc1.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/pmc1.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc2" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph > "$R/gpurun_out/pmc2.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/pmc2.log"; [ $rc -eq 0 ] || exit $rc
cd "$R"
python tools/pmc_summary.py $(find gpurun_out/pmc1 -name '*counter_collection.csv' | head -1) --title "PMC set 1: flagship wide step (1,835,008 envs, bench default)" -o gpurun_out/pmc1.md && \
python tools/pmc_summary.py $(find gpurun_out/pmc2 -name '*counter_collection.csv' | head -1) --title "PMC set 2: flagship wide step (1,835,008 envs, bench default)" -o gpurun_out/pmc2.md && cat gpurun_out/pmc1.md gpurun_out/pmc2.md
