#!/bin/bash
# round 3: full GPU suite (ws default), stamps + PMC of the production ws kernel, then the multi-rank
# rehearsals on one card (scripts/gpu_r3o.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-episode > gpurun_out/r3p_bench.log 2>&1 && echo "bench: $(tail -1 gpurun_out/r3p_bench.log | cut -c100-200)" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3p_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r3p_suite.log; exit 1; }
tail -2 gpurun_out/r3p_suite.log
timeout -k 10 120 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r3p_stamps_ws.md \
  > gpurun_out/r3p_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r3p_stamps.log; exit 1; }
cat gpurun_out/r3p_stamps_ws.md
rm -rf gpurun_out/r3p_pmc1 gpurun_out/r3p_pmc2
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/r3p_pmc1" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph --no-episode > "$R/gpurun_out/r3p_pmc1.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo PMC1_FAIL; exit $rc; }
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/r3p_pmc2" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph --no-episode > "$R/gpurun_out/r3p_pmc2.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo PMC2_FAIL; exit $rc; }
cd "$R"
python tools/pmc_summary.py $(find gpurun_out/r3p_pmc1 -name '*counter_collection.csv' | head -1) --title "PMC set 1: ws step kernel (1,835,008 envs)" -o gpurun_out/r3p_pmc1.md && \
python tools/pmc_summary.py $(find gpurun_out/r3p_pmc2 -name '*counter_collection.csv' | head -1) --title "PMC set 2: ws step kernel (1,835,008 envs)" -o gpurun_out/r3p_pmc2.md && echo PMC_OK
bash scripts/gpu_r3o.sh
