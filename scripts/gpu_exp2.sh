#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_api.py -x -v --timeout 120 --timeout-method thread > gpurun_out/exp2_tests.log 2>&1; rc=$?
tail -15 gpurun_out/exp2_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/train_overhead.py > gpurun_out/ovh2.log 2>&1 || { tail gpurun_out/ovh2.log; exit 1; }
head -3 gpurun_out/ovh2.log
