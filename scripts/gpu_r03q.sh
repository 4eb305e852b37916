#!/bin/bash
# Round 3: fixed per-launch cost of the group sweep (the strong-scaling bound):
# kernel trace of 1/1, 1/8, 1/64 shards (sample launch + sweep launch each),
# then instruction-cache counters per dispatch.
set -u
mkdir -p gpurun_out/q
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/q/avail.txt 2>&1
echo "list rc=$? $(grep -o 'SQC_ICACHE[A-Z_]*' gpurun_out/q/avail.txt | sort -u | tr '\n' ' ')"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q/trace -o run -- python3 scripts/shard_ablate.py 0 > gpurun_out/q/trace.log 2>&1
rc=$?; echo "trace rc=$rc $(grep ablate gpurun_out/q/trace.log)"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/q/ic -o run -- python3 scripts/shard_ablate.py 0 > gpurun_out/q/ic.log 2>&1
rc=$?; echo "icache rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/q/ic.log; exit $rc; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/q/sq -o run -- python3 scripts/shard_ablate.py 0 > gpurun_out/q/sq.log 2>&1
rc=$?; echo "sq rc=$rc"
exit $rc
