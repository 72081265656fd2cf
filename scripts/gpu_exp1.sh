#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python scripts/tune_dot.py 1024 p0,p20 > gpurun_out/exp1.log 2>&1; rc=$?
cat gpurun_out/exp1.log; exit $rc
