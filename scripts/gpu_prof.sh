#!/bin/bash
# Profiling call: phase stamps + PMC counters of the flagship step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python tools/stamp_qstep.py --out gpurun_out/stamps.md > gpurun_out/stamps.log 2>&1
rc=$?; cat gpurun_out/stamps.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
rocprofv3 -L > gpurun_out/counters_all.txt 2>&1 || true
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-graph > "$R/gpurun_out/prof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/prof.log"; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc1" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph > "$R/gpurun_out/pmc1.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/pmc1.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/pmc2" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph > "$R/gpurun_out/pmc2.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/pmc2.log"; exit $rc
