#!/bin/bash
# Round 3: kernel trace of the R=64 n=7 bench step (seed pre-pass timing).
set -u
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r03o_trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/r03o_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
