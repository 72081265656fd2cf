#!/bin/bash
# Rehearse the N>1 bench path with 2 ranks on ONE GPU (gloo, since RCCL needs distinct
# devices; kge.sharded stages device tensors through host memory for gloo); the real
# N=1/2/4/8 RCCL runs are the driver's.
set -o pipefail
mkdir -p gpurun_out
export KGE_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-c5 > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err
echo "exit $?"; cat gpurun_out/bench_n2_gloo.json; tail -5 gpurun_out/bench_n2_gloo.err
