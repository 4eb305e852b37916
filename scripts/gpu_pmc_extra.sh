#!/bin/bash
# One extra PMC pass over a short bench run: PMC="ctr ctr ..." (<= 8 SQ counters), TAG names the output.
set -u
mkdir -p gpurun_out/pmcx
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmcx/${TAG:-x} -o run -- $B > gpurun_out/pmcx/${TAG:-x}.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/pmcx/${TAG:-x}.log
exit $rc
