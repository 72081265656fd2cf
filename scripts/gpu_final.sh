#!/bin/bash
# Round-end evidence: the round script (tests, smoke, bench, rocprof of the bench), the C5
# shard extra, and a rocprof of the replayed 1vsAll training step.
set -o pipefail
bash scripts/gpu_round.sh || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu --c5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "c5 failed"; tail gpurun_out/bench_c5.err; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_train -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_train.py > $GRAFT_REPO_ROOT/gpurun_out/prof_train.log 2>&1 || { echo "train prof failed"; exit 1; }
echo done
