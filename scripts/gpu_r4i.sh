#!/bin/bash
# round 3 final flagship checkpoint: GPU suite, bench at the driver's args, stamps, PMC sets, kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4i_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r4i_suite.log; exit 1; }
tail -1 gpurun_out/r4i_suite.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4i_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r4i_bench.log; exit 1; }
tail -1 gpurun_out/r4i_bench.log | cut -c1-300
timeout -k 10 60 python -u __graft_entry__.py smoke > gpurun_out/r4i_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r4i_smoke.log; exit 1; }
timeout -k 10 150 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r4i_stamps_ws.md \
  > gpurun_out/r4i_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r4i_stamps.log; exit 1; }
rm -rf gpurun_out/r4i_pmc1 gpurun_out/r4i_pmc2 gpurun_out/r4i_prof
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/r4i_pmc1" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph --no-episode > "$R/gpurun_out/r4i_pmc1.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo PMC1_FAIL; exit $rc; }
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/gpurun_out/r4i_pmc2" -o pmc -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-graph --no-episode > "$R/gpurun_out/r4i_pmc2.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo PMC2_FAIL; exit $rc; }
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4i_prof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 5 --no-episode > "$R/gpurun_out/r4i_prof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { echo PROF_FAIL; exit $rc; }
cd "$R"
python tools/pmc_summary.py $(find gpurun_out/r4i_pmc1 -name '*counter_collection.csv' | head -1) --title "PMC set 1: ws step kernel, round-3 final (1,835,008 envs)" -o gpurun_out/r4i_pmc1.md && \
python tools/pmc_summary.py $(find gpurun_out/r4i_pmc2 -name '*counter_collection.csv' | head -1) --title "PMC set 2: ws step kernel, round-3 final (1,835,008 envs)" -o gpurun_out/r4i_pmc2.md && echo PMC_OK
cat gpurun_out/r4i_pmc2.md | head -16
