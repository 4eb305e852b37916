#!/bin/bash
# Extra PMC passes over a short bench run: PASSES="ctr ctr ...;ctr ctr ..." (one rocprofv3 run each).
set -u
mkdir -p gpurun_out/pmcx
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
IFS=';' read -ra PS <<< "$PASSES"
i=0
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcx/p$i -o run -- $B > gpurun_out/pmcx/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmcx/p$i.log; exit $rc; }
done
exit 0
