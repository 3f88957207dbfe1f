#!/bin/bash
# per-phase stamps of the ws kernel at the bench batch: u16 tick windows vs fp32 windows
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/stamp_qstep.py --kernel ws --envs 1835008 --bank16 auto --out $O/stamps_u16.md > $O/u16.log 2>&1 || { tail -20 $O/u16.log; exit 1; }
timeout -k 10 300 python tools/stamp_qstep.py --kernel ws --envs 1835008 --bank16 off --out $O/stamps_fp32.md > $O/fp32.log 2>&1 || { tail -20 $O/fp32.log; exit 1; }
cat $O/stamps_u16.md $O/stamps_fp32.md
