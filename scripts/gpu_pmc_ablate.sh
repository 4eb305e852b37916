#!/bin/bash
# PMC of the group kernel under ablation masks (timing diagnostics, ablation
# library): MASKS="0 15349" bash scripts/gpu_pmc_ablate.sh
set -u
mkdir -p gpurun_out/pmca
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export BOTE_LIB_PATH=fantoch_amd/lib_abl/libbote_hip.so
P=${PMC:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"}
for M in ${MASKS:-0}; do
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmca/m$M -o run -- python3 scripts/ablate.py $M > gpurun_out/pmca/m$M.log 2>&1
  rc=$?; echo "mask $M rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmca/m$M.log; exit $rc; }
  python3 - "$M" <<'PY'
import csv, sys, collections
m = sys.argv[1]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f"gpurun_out/pmca/m{m}/run_counter_collection.csv")):
    if "sweep_group" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
steps = 621216192 / 64
print("mask", m, " ".join(f"{k}={sum(v)/len(v)/steps:.1f}/step" for k, v in sorted(acc.items())))
PY
done
