#!/bin/bash
# rocprof kernel breakdowns of the C3 (KvsAll DistMult) and C4 (NS RotatE) training steps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/prof_train.py distmult KvsAll > $GRAFT_REPO_ROOT/gpurun_out/prof_c3.log 2>&1 || { echo "c3 failed"; tail $GRAFT_REPO_ROOT/gpurun_out/prof_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/prof_ns.py > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1 || { echo "c4 failed"; tail $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/dev/prof_train.py distmult KvsAll 2>&1 | grep step
timeout -k 10 120 python scripts/dev/prof_ns.py 2>&1 | grep -i "step\|ms"
