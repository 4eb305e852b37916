#!/bin/bash
# TEST INFRASTRUCTURE — regenerates the oracle-pinned sweep fixtures under
# tests/golden/ (CPU only, hours of work: run in the background, resumable).
#   1. R=128 n=6: nine 10^6-rank windows, eight of them straddling a colex
#      boundary C(m,6) where every member changes (first/last ranks included);
#   2. R=64 n=7: all 621,216,192 ranks (bench workload).
set -euo pipefail
cd "$(dirname "$0")/.."
T=${THREADS:-8}
if [ ! -f tests/golden/syn_r128n6_windows.json ]; then
for b in 0 3338380 49563860 300000200 1191552400 2141351635 3652245460 5168879425 5422611200; do
  python scripts/oracle_full_sweep.py --workload r128n6 --threads "$T" --chunk 1000000 \
    --rank-begin "$b" --rank-end $((b + 1000000)) --name "win_r128n6_$b"
done
python - <<'EOF'
import glob, json, os
ws = []
for p in sorted(glob.glob("tests/golden/win_r128n6_*.json"), key=lambda p: int(p.rsplit("_", 1)[1][:-5])):
    ws.append(json.load(open(p)))
    os.remove(p)
json.dump({"what": "oracle sweeps of 10^6-rank windows of the synthetic R=128 planet, n=6",
           "generator": "scripts/oracle_fixtures.sh", "windows": ws}, open("tests/golden/syn_r128n6_windows.json", "w"))
EOF
fi
python scripts/oracle_full_sweep.py --workload r64n7 --threads "$T" --chunk 4194304
