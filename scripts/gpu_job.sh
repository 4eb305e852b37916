#!/bin/bash
# One parameterised GPU job (one gpurun call): the steps named in STEPS, in
# order, each under its own time limit; the job stops at the first step that
# fails (a fault, an abort or a time limit ends it: nothing else runs on the GPU).
#
#   STEPS="smoke tests bench profile" TAG=r04a bash scripts/gpu_job.sh
#
# Steps (outputs under gpurun_out/$TAG/):
#   smoke    __graft_entry__.py (smoke on cuda:0)
#   tests    pytest -m gpu over TEST_FILES (default tests/; PYTEST_EXPR: a -k expression)
#   bench    bench.py with the CPU baseline, for each workload in BWLS (default WLS)
#   ab       A/B timing of library variants: VARIANTS="default lib_x ..." (lib_x:
#            fantoch_amd/lib_x/libbote_hip.so, scripts/build_variant.sh), REPS
#            rounds interleaved, for each workload in WLS; AB_SKIP=1 passes
#            --skip-fixture-check (diagnostics while a fixture is re-pinned)
#   profile  rocprofv3 kernel trace + stats, then the PMC passes of
#            scripts/summarize_profile.py, of bench.py on each workload in
#            PWLS (default WL), to gpurun_out/$TAG/<workload>/ (PSTEPS steps
#            after PWARM warm-up steps, default 3 and 1; the summary leaves
#            the warm-up launches out of its averages)
#   summarize  scripts/summarize_profile.py of the profile step's runs (on the box, before a bench step)
#   pin      config 5's full-size regression pin (scripts/pin_r128n6.py)
#   trace    rocprofv3 kernel trace + stats (no counters) of bench.py for each workload in TWLS
#   pmc      extra PMC passes: PASSES="ctr ...;ctr ..." over bench.py BENCH_ARGS
#   shardsteps  scripts/shard_steps.py (a shard's step: wall, kernel, outside) per VARIANTS, + a trace
#   shards   kernel trace of scripts/shard_ablate.py (per-dispatch cost of shards)
#   ablate   scripts/ablate.py masks ABL on the -DBOTE_ABLATION library (lib_abl)
#   pstats   scripts/pathstats.py on the -DBOTE_PATHSTATS library (lib_pstats), for each workload in WLS
#   oracle   the CPU oracle over R=64 n=7 chunks from ORACLE_BEGIN for
#            ORACLE_SECONDS (scripts/oracle_full_sweep.py --partial; state to
#            gpurun_out/$TAG/oracle_chunks.jsonl, merged into the fixture here)
set -u
TAG=${TAG:-job}
O=gpurun_out/$TAG
mkdir -p "$O"
export PYTHONUNBUFFERED=1
WLS=${WLS:-r64n7}

fail() { echo "$1 rc=$2"; [ -f "$3" ] && tail -15 "$3"; exit "$2"; }

step_smoke() {
  timeout -k 10 300 python -u __graft_entry__.py > "$O/smoke.log" 2>&1 || fail smoke $? "$O/smoke.log"
  echo "smoke ok: $(tail -1 "$O/smoke.log")"
}

step_tests() {
  local sel=(-m gpu)
  [ -n "${PYTEST_EXPR:-}" ] && sel=(-m gpu -k "$PYTEST_EXPR")
  timeout -k 10 1100 python -u -m pytest ${TEST_FILES:-tests/} "${sel[@]}" -x -v --timeout 400 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || fail tests $? "$O/gpu_tests.log"
  echo "tests ok: $(tail -1 "$O/gpu_tests.log")"
}

step_bench() {
  for wl in ${BWLS:-$WLS}; do
    timeout -k 10 400 python -u bench.py --workload "$wl" --steps "${BSTEPS:-20}" --warmup 2 ${BENCH_ARGS:-} \
      > "$O/bench_$wl.log" 2>&1 || fail "bench $wl" $? "$O/bench_$wl.log"
    echo "bench $wl: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"fixture": "[^"]*' "$O/bench_$wl.log" | tr '\n' ' ')"
  done
}

step_ab() {
  local skip=""
  [ "${AB_SKIP:-0}" = 1 ] && skip="--skip-fixture-check"
  for r in $(seq 1 "${REPS:-2}"); do
    for wl in $WLS; do
      for V in ${VARIANTS:-default}; do
        if [ "$V" = default ]; then unset BOTE_LIB_PATH; else export BOTE_LIB_PATH=fantoch_amd/$V/libbote_hip.so; fi
        timeout -k 10 300 python -u bench.py --workload "$wl" --steps "${ABSTEPS:-10}" --warmup 2 --no-cpu-baseline $skip \
          > "$O/ab_${wl}_${V}_$r.log" 2>&1 || fail "ab $wl $V" $? "$O/ab_${wl}_${V}_$r.log"
        echo "ab $wl $V #$r: $(grep -o '"kernel_ms_avg": [0-9.]*\|"ms_per_step": [0-9.]*\|"valid": [0-9]*\|"digest": [0-9]*' "$O/ab_${wl}_${V}_$r.log" | tr '\n' ' ')"
      done
    done
  done
  unset BOTE_LIB_PATH
}

step_profile() {
  export TMPDIR=/tmp
  local wl
  for wl in ${PWLS:-${WL:-r64n7}}; do
    local P="$O/$wl"
    mkdir -p "$P"
    local B="python3 bench.py --steps ${PSTEPS:-3} --warmup ${PWARM:-1} --no-cpu-baseline --workload $wl ${BENCH_ARGS:-}"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace" -o run -- $B \
      > "$P/trace.log" 2>&1 || fail "trace $wl" $? "$P/trace.log"
    echo "trace $wl ok"
    local P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
    local P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
    local i=0
    for Q in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
      i=$((i + 1))
      timeout -s KILL 240 rocprofv3 --pmc $Q --output-format csv -d "$P/pmc$i" -o run -- $B \
        > "$P/pmc$i.log" 2>&1 || fail "pmc$i $wl" $? "$P/pmc$i.log"
      echo "pmc$i $wl ok"
    done
  done
}

step_summarize() {  # the profile step's summaries on the box (profiles/pmc.json, traffic.json), so that a bench step
  # after it in the same job quotes the same build's VALU issue and traffic; re-run it here on return
  local wl
  for wl in ${PWLS:-${WL:-r64n7}}; do
    timeout -k 10 120 python3 scripts/summarize_profile.py "$TAG/$wl" "${wl}_n1" > "$O/summarize_$wl.log" 2>&1 \
      || fail "summarize $wl" $? "$O/summarize_$wl.log"
    echo "summarize $wl ok"
  done
}

step_pin() {  # config 5's full-size regression pin (scripts/pin_r128n6.py) to gpurun_out/$TAG/syn_r128n6_pin.json
  timeout -k 10 600 python3 -u scripts/pin_r128n6.py "$O/syn_r128n6_pin.json" > "$O/pin.log" 2>&1 || fail pin $? "$O/pin.log"
  echo "pin: $(tail -1 "$O/pin.log")"
}

step_trace() {  # kernel trace + stats only (no PMC), for each workload in TWLS
  export TMPDIR=/tmp
  local wl
  for wl in ${TWLS:-r64n7}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$wl" -o run -- \
      python3 bench.py --steps "${TSTEPS:-5}" --warmup 1 --no-cpu-baseline --workload "$wl" ${BENCH_ARGS:-} \
      > "$O/trace_$wl.log" 2>&1 || fail "trace $wl" $? "$O/trace_$wl.log"
    echo "trace $wl: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"step_overhead_ms": [0-9.]*' "$O/trace_$wl.log" | tr '\n' ' ')"
  done
}

step_pmc() {
  export TMPDIR=/tmp
  local B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
  local PS i=0
  IFS=';' read -ra PS <<< "$PASSES"
  for P in "${PS[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$O/pmcx$i" -o run -- $B \
      > "$O/pmcx$i.log" 2>&1 || fail "pmcx$i" $? "$O/pmcx$i.log"
    echo "pmcx$i ok"
  done
}

step_shards() {
  export TMPDIR=/tmp
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/shards" -o run -- \
    python3 scripts/shard_ablate.py ${SHARD_ARGS:-0} > "$O/shards.log" 2>&1 || fail shards $? "$O/shards.log"
  echo "shards ok: $(grep ablate "$O/shards.log" | tr '\n' ' ')"
}

step_shardsteps() {  # scripts/shard_steps.py per variant in VARIANTS, then a kernel trace of the default build
  export TMPDIR=/tmp
  for V in ${VARIANTS:-default}; do
    if [ "$V" = default ]; then unset BOTE_LIB_PATH; else export BOTE_LIB_PATH=fantoch_amd/$V/libbote_hip.so; fi
    timeout -k 10 180 python -u scripts/shard_steps.py 20 > "$O/shardsteps_$V.log" 2>&1 || fail "shardsteps $V" $? "$O/shardsteps_$V.log"
    echo "shardsteps $V: $(grep -o '"parts": [0-9]*\|"step_ms": [0-9.]*\|"outside_ms": [0-9.]*' "$O/shardsteps_$V.log" | tr '\n' ' ')"
  done
  unset BOTE_LIB_PATH
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/shardsteps_trace" -o run -- \
    python3 scripts/shard_steps.py 5 > "$O/shardsteps_trace.log" 2>&1 || fail shardsteps_trace $? "$O/shardsteps_trace.log"
  echo "shardsteps trace ok"
}

step_ablate() {
  BOTE_LIB_PATH=fantoch_amd/lib_abl/libbote_hip.so timeout -k 10 300 python -u scripts/ablate.py ${ABL:-0} \
    > "$O/ablate.log" 2>&1 || fail ablate $? "$O/ablate.log"
  grep -v amdgpu.ids "$O/ablate.log"
}

step_pstats() {
  for wl in $WLS; do
    BOTE_LIB_PATH=fantoch_amd/lib_pstats/libbote_hip.so timeout -k 10 300 python -u scripts/pathstats.py "$wl" \
      > "$O/pstats_$wl.json" 2> "$O/pstats_$wl.err" || fail "pstats $wl" $? "$O/pstats_$wl.err"
    echo "pstats $wl: $(tr -d '\n' < "$O/pstats_$wl.json" | cut -c1-600)"
  done
}

step_oracle() {
  timeout -k 10 $((${ORACLE_SECONDS:-600} + 200)) python -u scripts/oracle_full_sweep.py --workload r64n7 \
    --threads "${ORACLE_THREADS:-16}" --chunk 4194304 --partial --sweep-begin "${ORACLE_BEGIN:?}" \
    --time-limit "${ORACLE_SECONDS:-600}" --state "$O/oracle_chunks.jsonl" > "$O/oracle.log" 2>&1 \
    || fail oracle $? "$O/oracle.log"
  echo "oracle: $(tail -1 "$O/oracle.log")"
  if [ -n "${ORACLE_BEGIN2:-}" ]; then
    timeout -k 10 $((${ORACLE_SECONDS2:-300} + 200)) python -u scripts/oracle_full_sweep.py --workload r64n7 \
      --threads "${ORACLE_THREADS:-16}" --chunk 4194304 --partial --sweep-begin "$ORACLE_BEGIN2" \
      --time-limit "${ORACLE_SECONDS2:-300}" --state "$O/oracle_chunks.jsonl" > "$O/oracle2.log" 2>&1 \
      || fail oracle2 $? "$O/oracle2.log"
    echo "oracle2: $(tail -1 "$O/oracle2.log")"
  fi
}

for s in ${STEPS:?STEPS names the steps}; do
  "step_$s"
done
exit 0
