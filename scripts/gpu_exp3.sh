#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_losses.py tests/test_gpu_graph.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp3.log 2>&1 || { tail -30 gpurun_out/exp3.log; exit 1; }
tail -1 gpurun_out/exp3.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_train2 -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_train.py > $GRAFT_REPO_ROOT/gpurun_out/prof_train2.log 2>&1 || { echo "prof failed"; exit 1; }
cd $GRAFT_REPO_ROOT && timeout -k 10 200 python scripts/graph_probe.py 2>&1 | grep -v amdgpu.ids
