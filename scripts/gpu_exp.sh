#!/bin/bash
# One experiment call: GPU tests, distance-kernel A/B, contraction variants, C5 stress.
set -o pipefail
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/exp/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/exp/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/dist_ab.py 512 > gpurun_out/exp/dist.txt 2>&1 || { echo "dist failed"; tail gpurun_out/exp/dist.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/exp/dist.txt
timeout -k 10 200 python scripts/tune_dot.py 1024 "$1" > gpurun_out/exp/tune.txt 2>&1 || { echo "tune failed"; tail gpurun_out/exp/tune.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/exp/tune.txt
timeout -k 10 300 python scripts/stress_c5.py 574311 400 > gpurun_out/exp/stress.txt 2>&1 || { echo "stress failed"; tail gpurun_out/exp/stress.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/exp/stress.txt
