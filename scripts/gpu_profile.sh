#!/bin/bash
# rocprofv3: kernel trace + stats, then separate PMC passes (one block budget each).
set -u
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload ${WL:-r64n7}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG}_trace -o run -- $B > gpurun_out/prof/${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then tail -20 gpurun_out/prof/${TAG}_trace.log; exit $rc; fi
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d gpurun_out/prof/${TAG}_pmc$i -o run -- $B > gpurun_out/prof/${TAG}_pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; if [ $rc -ne 0 ]; then tail -20 gpurun_out/prof/${TAG}_pmc$i.log; exit $rc; fi
done
exit 0
