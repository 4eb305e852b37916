#!/bin/bash
# TEST INFRASTRUCTURE — regenerates the oracle-pinned sweep fixtures under
# tests/golden/ (CPU only, hours of work: run in the background, resumable).
#   1. the small fixtures: topk.json (tests/golden/make_golden.py topk);
#   2. the extended key set and the R=128 n=6 windows (boundary and seeded
#      random): topk_x.json, syn_r128n6_windows.json
#      (tests/golden/make_keys_golden.py);
#   3. R=64 n=7: all 621,216,192 ranks (bench workload), syn_r64n7_full.json.
set -euo pipefail
cd "$(dirname "$0")/.."
T=${THREADS:-8}
python tests/golden/make_golden.py topk
python tests/golden/make_keys_golden.py all --threads "$T"
python scripts/oracle_full_sweep.py --workload r64n7 --threads "$T" --chunk 4194304
