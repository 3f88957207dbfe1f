#!/bin/bash
# PMC passes over the serving kernel (1M-row batches, both gather paths), one run per counter set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/servepmc
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
i=0
for set in "$P1" "$P2"; do
  i=$((i + 1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/servepmc/p$i" -o run -- python3 "$R/benchmarks/bench_serve.py" --batches 1048576 --clients 2 --requests 5 > "$R/gpurun_out/servepmc/p$i.log" 2>&1 || exit $?
  cd "$R"
done
