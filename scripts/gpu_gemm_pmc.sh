#!/bin/bash
# PMC passes over one GEMM (TILE env: pp | 128 | hipblaslt; MNK env).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/gpmc
for t in ${TILES:-pp hipblaslt}; do
  cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA --output-format csv -d "$R/gpurun_out/gpmc/$t" -o run -- python3 "$R/tools/run_gemm_once.py" --tile $t --mnk ${MNK:-8192,8192,8192} > "$R/gpurun_out/gpmc/$t.log" 2>&1 || exit $?
  cd "$R"
done
