#!/bin/bash
# Fresh-container re-validation: the round script, then a rocprof kernel breakdown of the
# 1vsAll training step and the backward-GEMM sweep.
set -o pipefail
bash scripts/gpu_round.sh || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_train -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_train.py > $GRAFT_REPO_ROOT/gpurun_out/prof_train.log 2>&1 || { echo "train prof failed"; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/prof_train.log | tail -2
cd $GRAFT_REPO_ROOT && timeout -k 10 200 python scripts/tune_bwd.py 2048 16 0,2,3 > gpurun_out/tune_bwd.log 2>&1 || { echo "tune_bwd failed"; exit 1; }
cat gpurun_out/tune_bwd.log
