#!/bin/bash
# Contraction-kernel experiment: interleaved timing of variants, clock probe, PMC traffic.
# usage: bash scripts/dev/gpu_tune.sh "<variants for tune_dot>" "<clock variants>" "<pmc variants>"
set -o pipefail
mkdir -p gpurun_out/tune
export TMPDIR=/tmp
timeout -k 10 240 python scripts/dev/tune_dot.py 1024 "$1" > gpurun_out/tune/tune.txt 2>&1 || { echo "tune failed"; tail gpurun_out/tune/tune.txt; exit 1; }
cat gpurun_out/tune/tune.txt
if [ -n "$2" ]; then
  timeout -k 10 120 python scripts/dev/clock_probe.py "$2" > gpurun_out/tune/clock.txt 2>&1 || { echo "clock failed"; tail gpurun_out/tune/clock.txt; exit 1; }
  cat gpurun_out/tune/clock.txt
fi
cd /tmp
for v in $3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tune/pmc_${v}_$ctr -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/tune_one.py $v > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/tune/pmc_err.txt || { echo "pmc $v $ctr failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/tune/pmc_err.txt; exit 1; }
  done
done
cd $GRAFT_REPO_ROOT
for dir in gpurun_out/tune/pmc_*/; do echo "$dir"; python3 scripts/dev/pmc_summary.py "$dir" score_dot 2>&1 | tail -3; done
