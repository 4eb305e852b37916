#!/bin/bash
# Ablation timings + one SQ counter pass of the default sweep kernel (R=64 n=7).
set -u
mkdir -p gpurun_out/qp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u scripts/ablate.py ${ABL:-0 1 4 8 16 31} > gpurun_out/qp/ablate.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/qp/ablate.log; [ $rc -ne 0 ] && exit $rc
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/qp/pmc1 -o run -- $B > gpurun_out/qp/pmc1.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/qp/pmc1.log
exit $rc
