#!/bin/bash
# PMC passes (kernel-trace only) over the backward-GEMM sweep (dT written: variant 2, dQ: 0)
# and the forward contraction, for an issue/stall breakdown.
set -o pipefail
mkdir -p gpurun_out/pmcb
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_CMD_FIFO_FULL"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcb/b$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/tune_bwd.py 2048 8 0,2 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/pmcb/errb$i.txt || { echo "pass b$i failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmcb/errb$i.txt; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcb/f$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/tune_dot.py 1024 p0 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/pmcb/errf$i.txt || { echo "pass f$i failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmcb/errf$i.txt; exit 1; }
done
echo done
