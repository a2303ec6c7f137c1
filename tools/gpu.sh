#!/bin/bash
# The one GPU-box runner: `tools/gpu.sh TAG STEP [STEP ...]`, e.g.
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh r6a tests smoke bench profile sq drop_in'
# Every step that touches the GPU runs under its own time limit; the steps run in order and the script stops at the
# first failure (crash, abort, timeout or failed test), so nothing more runs on a GPU in a bad state.  Output goes to
# gpurun_out/TAG/.  Steps:
#   tests            pytest -m gpu (the driver's suite), log pytest_gpu.log, parity_report.json copied
#   smoke            __graft_entry__.smoke()
#   bench            the headline bench line (bench.py defaults; BENCH_ARGS appended) -> bench_b32.json
#   profile          rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE PMC passes (tools/profile_round.sh)
#   sq               the SQ / GRBM counter passes behind tools/sq_table.py (tools/pmc_pass.sh)
#   drop_in          bench lines for batch 1, batch 4, the YODAS2-style and MLS-style workloads
#   ab               tools/ab_libs.sh (LIBS, ROUNDS, STEPS, KEYS, BENCH_ARGS from the environment)
#   taps             tools/race_taps.py: engine A's stage taps vs A alone while a clone loads the GPU (REPS, 300)
#   race             tools/race_probe.py: codes of two engines encoding at once vs one alone
#   pk_probe         tools/pk_probe.hip: each packed-f32 operand form vs scalar, idle and under concurrent load
#   bits             tools/lib_codes.py for each ab/libmimi_hip_<name>.so in BITS_LIBS and the in-tree library, then
#                    tools/cmp_codes.py: codes and every stage tap bitwise against the first of BITS_LIBS
#   gloo2            the N-rank bench path rehearsed on this box: --gpus 2 over gloo, both ranks sharing its GPU
#                    (the line must list both ranks on one PCI bus and say `sharing`)
#   b:NAME:ARGS      one bench run with ARGS (spaces as '+'), -> bench_NAME.json
#   t:FILE          one GPU test file (tests/FILE), log t_FILE.log
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${1:?usage: tools/gpu.sh TAG STEP...}
shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"

fail() { echo "step $1 failed (rc=$2)"; [ -f "$3" ] && tail -20 "$3"; exit 1; }

bench_line() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --cpu-baseline-seconds 0 "$@" --json-out "$O/bench_$name.json" \
    > "$O/bench_$name.log" 2>&1 || fail "bench $name" $? "$O/bench_$name.log"
  python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', d['value'], d['ms_per_step'])"
}

for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
        -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1 || fail tests $? "$O/pytest_gpu.log"
      tail -1 "$O/pytest_gpu.log"
      cp gpurun_out/parity_report.json "$O/parity_report.json" 2>/dev/null || true ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail smoke $? "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} --json-out "$O/bench_b32.json" > "$O/bench_b32.log" 2>&1 \
        || fail bench $? "$O/bench_b32.log"
      python3 -c "import json; d=json.load(open('$O/bench_b32.json')); print('b32', d['value'], d['ms_per_step'], d['roofline']['frac'])" ;;
    profile)
      TAG=$TAG STEPS=10 timeout -k 10 900 bash tools/profile_round.sh > "$O/profile_round.log" 2>&1 \
        || fail profile $? "$O/profile_round.log"
      echo "profile ok" ;;
    sq)
      PASSES="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE;SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE" \
        TAG=${TAG}_sq timeout -k 10 400 bash tools/pmc_pass.sh > "$O/sq.log" 2>&1 || fail sq $? "$O/sq.log"
      echo "sq ok" ;;
    drop_in)
      bench_line b1 --batch 1 --no-f32-mode
      bench_line b4 --batch 4 --no-f32-mode
      bench_line yodas2 --workload yodas2 --steps 12 --warmup 2
      bench_line mls --workload mls --steps 8 --warmup 1 ;;
    ab)
      timeout -k 10 1000 bash tools/ab_libs.sh > "$O/ab.log" 2>&1 || fail ab $? "$O/ab.log"
      cat "$O/ab.log" ;;
    taps)
      timeout -k 10 300 python -u tools/race_taps.py ${REPS:-300} nocontrols > "$O/taps.log" 2>&1 \
        || fail taps $? "$O/taps.log"
      echo "taps: $(grep -c '^loaded' "$O/taps.log") of ${REPS:-300} loaded reps differ, $(grep -c '^idle' "$O/taps.log") idle" ;;
    race)
      timeout -k 10 300 python -u tools/race_probe.py 24 all > "$O/race.log" 2>&1 || fail race $? "$O/race.log"
      grep setting "$O/race.log" ;;
    pk_probe)
      mkdir -p tools/bin
      /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/pk_probe.hip -o tools/bin/pk_probe > "$O/pk_build.log" 2>&1 \
        || fail pk_build $? "$O/pk_build.log"
      timeout -k 10 300 tools/bin/pk_probe ${LAUNCHES:-40} > "$O/pk_probe.log" 2>&1 || fail pk_probe $? "$O/pk_probe.log"
      cat "$O/pk_probe.log" ;;
    bits)
      for v in ${BITS_LIBS:?BITS_LIBS} new; do
        if [ $v = new ]; then unset MIMI_HIP_LIB; else export MIMI_HIP_LIB=$R/ab/libmimi_hip_$v.so; fi
        timeout -k 10 300 python -u tools/lib_codes.py ${TAG}_$v > "$O/bits_$v.log" 2>&1 || fail "bits $v" $? "$O/bits_$v.log"
      done
      unset MIMI_HIP_LIB
      ref=${BITS_LIBS%% *}
      python3 tools/cmp_codes.py ${TAG}_$ref $(for v in ${BITS_LIBS#$ref} new; do echo ${TAG}_$v; done) > "$O/bits_cmp.txt" 2>&1
      rc=$?; grep -c "bitwise equal" "$O/bits_cmp.txt"; grep -v "bitwise equal" "$O/bits_cmp.txt" | head -20
      [ $rc -eq 0 ] || fail bits_cmp $rc "$O/bits_cmp.txt" ;;
    gloo2)
      MIMI_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 \
        --cpu-baseline-seconds 0 --no-f32-mode --json-out "$O/bench_gloo2.json" > "$O/bench_gloo2.log" 2>&1 \
        || fail gloo2 $? "$O/bench_gloo2.log"
      python3 -c "import json; d=json.load(open('$O/bench_gloo2.json')); print('gloo2', d['value'], d['dist'], [(r['rank'], r['pci_bus']) for r in d['ranks']])" ;;
    t:*)
      f=${step#t:}
      timeout -k 10 600 python -u -m pytest "tests/$f" -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$O/t_$f.log" 2>&1 || fail "test $f" $? "$O/t_$f.log"
      tail -1 "$O/t_$f.log" ;;
    b:*)
      spec=${step#b:}; name=${spec%%:*}; args=${spec#*:}
      bench_line "$name" ${args//+/ } ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
