#!/bin/bash
# PMC of the final flagship step (ws kernel + optimizer pass) at the bench batch: MFMA busy, waits, HBM bytes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5pmcf}
mkdir -p $D
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES FETCH_SIZE --output-format csv -d $D/pmc1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-episode --no-graph > $D/pmc1.log 2>&1 || exit 1
f=$(find $D/pmc1 -name "*counter_collection.csv" | head -1); echo $f
python3 tools/pmc_summary.py $f --kernels qstep_ws,reduce_optim --title "PMC: final round-5 flagship step, 1,835,008 envs" -o $D/pmc_final.md && cat $D/pmc_final.md
