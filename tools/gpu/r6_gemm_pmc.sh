#!/bin/bash
# PMC of the ping-pong GEMM at the act step's shape: production (0) and the no-staging / MFMA-only / no-MFMA ablations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gemmpmc
mkdir -p $O
for v in 0 1 2 3; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $O/p1_$v -o run -- tools/ubench/gemm_lab.bin pmc $v > $O/p1_$v.log 2>&1 || { tail $O/p1_$v.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p2_$v -o run -- tools/ubench/gemm_lab.bin pmc $v > $O/p2_$v.log 2>&1 || { tail $O/p2_$v.log; exit 1; }
done
ls -R $O | head -40
