#!/bin/bash
# One GPU visit, in phases (each GPU step has its own limit; a fault, abort or
# time-out ends the script -- nothing more runs on the GPU in that call).
#   PHASE=check      pytest -m gpu, smoke(), bench.py (default line + A/B lines)
#   PHASE=ab         bench.py A/B lines only (AB="name:ENV=v:--arg%value ...")
#   PHASE=profile    rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes of bench.py (LAYOUT=NMC|MNC)
#   PHASE=benchprof  rocprofv3 of EXACTLY the driver's bench command + FETCH / WRITE passes
#   PHASE=configs    kernel traces of tools/bench_configs.py + FETCH / WRITE of the wide config
#   PHASE=xgb        the same for the XGB member (tools/bench_configs.py --only 7)
#   PHASE=mpmc       PMC passes over the member kernels (tools/members_pmc.py)
#   PHASE=small      kernel traces of the small-pool configs + PMC passes of one (tools/small_probe.py)
#   PHASE=c5         rocprofv3 of the full C5 job (tools/bench_c5.py) + PMC passes at 12M items
#   PHASE=c5ab       the C5 job at 12M items per library build (ABLIBS="base x"), alternating
#   PHASE=smallab    small-pool configs under rocprofv3 per library build (LIBS="base reg"), alternating
#   PHASE=debug      pytest -m gpu on the debug build (CE_DASSERT device bounds checks)
#   PHASE=phase      per-block phase stamps of C3 on the diagnostic build (make phase)
#   PHASE=firstcall  first-call latency per library build (tools/first_call.py)
#   PHASE=c3drain    rocprofv3 of tools/c3_drain_probe.hip (configs[2] reads only: the load floor)
#   PHASE=c5probe    tools/c5_probe.py per library build (LIBS="base x"), alternating (wide stream: iid vs rising pools)
#   PHASE=gather     tools/gather_probe.py + FETCH / WRITE passes of the shuffled-frames kernel
#   PHASE=framesab   tools/gather_probe.py per library build (LIBS="base x"), alternating
#   PHASE=scale      tools/scale_proxy.py (per-rank proxies; world-1 RCCL step eager vs HIP graph)
#   PHASE=tests      selected GPU tests (TESTS=files, TESTK=-k expression, PYTEST_ARGS=...)
# Usage (from the repo root): gpurun -- 'PHASE=check bash tools/gpu_round.sh'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
LOG=$OUT/steps.log
echo "start $PHASE $(date)" >> "$LOG"
step() {  # $1 = status, $2 = name; 1 = test failures (keep going), anything else stops
  echo "$2: $1" >> "$LOG"
  case "$1" in 0|1) return 0 ;; *) echo "STOP after $2 ($1)" >> "$LOG"; exit "$1" ;; esac
}
bench() {  # $1 = name, rest = env/args
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  step $? "bench $name"
}
case "$PHASE" in
check)
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1
  step $? pytest
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  step $? smoke
  bench nmc python bench.py ${BENCH_ARGS}
  for v in ${AB}; do  # AB="name:ENV=val,ENV2=val:args ..."
    IFS=: read -r n e a <<< "$v"
    bench "$n" ${e//,/ } python bench.py --no-cpu-baseline ${a//\%/ }
  done
  ;;
ab)  # A/B lines only: AB="name:ENV=v,ENV2=v:--arg%value ..." (% stands for a space)
  for v in ${AB}; do
    IFS=: read -r n e a <<< "$v"
    bench "$n" ${e//,/ } python bench.py --no-cpu-baseline ${a//\%/ }
  done
  ;;
profile)
  LAYOUT=${LAYOUT:-NMC}
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof/trace_$LAYOUT" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --layout "$LAYOUT" > "$OUT/prof_trace_$LAYOUT.log" 2>&1
  step $? "trace $LAYOUT"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/fetch_$LAYOUT" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --layout "$LAYOUT" > "$OUT/prof_fetch_$LAYOUT.log" 2>&1
  step $? "fetch $LAYOUT"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/write_$LAYOUT" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --layout "$LAYOUT" > "$OUT/prof_write_$LAYOUT.log" 2>&1
  step $? "write $LAYOUT"
  ;;
benchprof)  # rocprofv3 kernel trace of EXACTLY the driver's bench command (its JSON line on stdout)
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof/bench_exact" -o run --output-format csv -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_exact.json" 2> "$OUT/bench_exact.err"
  step $? "trace bench exact"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/fetch_NMC" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof_fetch_NMC.log" 2>&1
  step $? "fetch NMC"
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/write_NMC" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof_write_NMC.log" 2>&1
  step $? "write NMC"
  ;;
configs)  # kernel-trace stats of every secondary config + FETCH/WRITE passes of the wide one
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof/configs" -o run --output-format csv -- python3 "$ROOT/tools/bench_configs.py" > "$OUT/prof_configs.log" 2>&1
  step $? "trace configs"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/fetch_wide" -o run --output-format csv -- python3 "$ROOT/tools/bench_configs.py" --only 4 > "$OUT/prof_fetch_wide.log" 2>&1
  step $? "fetch wide"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/write_wide" -o run --output-format csv -- python3 "$ROOT/tools/bench_configs.py" --only 4 > "$OUT/prof_write_wide.log" 2>&1
  step $? "write wide"
  ;;
xgb)  # kernel-trace stats + FETCH_SIZE pass of the XGB member (bench_configs --only 7)
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof/xgb" -o run --output-format csv -- python3 "$ROOT/tools/bench_configs.py" --only 7 > "$OUT/prof_xgb.log" 2>&1
  step $? "trace xgb"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/fetch_xgb" -o run --output-format csv -- python3 "$ROOT/tools/bench_configs.py" --only 7 > "$OUT/prof_fetch_xgb.log" 2>&1
  step $? "fetch xgb"
  ;;
mpmc)  # PMC passes over the member kernels (tools/members_pmc.py): SQ occupancy/stall/VALU/LDS, TA/TCP gather load
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d "$OUT/prof/mpmc_sq" -o run --output-format csv -- python3 "$ROOT/tools/members_pmc.py" ${MPMC_ARGS} > "$OUT/mpmc_sq.log" 2>&1
  step $? "mpmc sq"
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum -d "$OUT/prof/mpmc_ta" -o run --output-format csv -- python3 "$ROOT/tools/members_pmc.py" ${MPMC_ARGS} > "$OUT/mpmc_ta.log" 2>&1
  step $? "mpmc ta"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/prof/mpmc_sq2" -o run --output-format csv -- python3 "$ROOT/tools/members_pmc.py" ${MPMC_ARGS} > "$OUT/mpmc_sq2.log" 2>&1
  step $? "mpmc sq2"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM -d "$OUT/prof/mpmc_lds" -o run --output-format csv -- python3 "$ROOT/tools/members_pmc.py" ${MPMC_ARGS} > "$OUT/mpmc_lds.log" 2>&1
  step $? "mpmc lds"
  ;;
small)  # single-block / small-pool configs: one kernel trace per config + PMC passes of configs[2] (dense)
  cd /tmp
  for c in ${CFGS:-c1 c2hc c2mix c3 c3r}; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof/${TAG}small_$c" -o run --output-format csv -- python3 "$ROOT/tools/small_probe.py" $c 200 > "$OUT/${TAG}small_$c.log" 2>&1
    step $? "trace $TAG$c"
  done
  P=${PMCCFG:-c3}
  if [ "$P" != none ]; then
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/${TAG}pmc_fetch" -o run --output-format csv -- python3 "$ROOT/tools/small_probe.py" $P 20 > "$OUT/${TAG}pmc_fetch.log" 2>&1
  step $? "${TAG}pmc fetch"
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/${TAG}pmc_write" -o run --output-format csv -- python3 "$ROOT/tools/small_probe.py" $P 20 > "$OUT/${TAG}pmc_write.log" 2>&1
  step $? "${TAG}pmc write"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/prof/${TAG}pmc_sq" -o run --output-format csv -- python3 "$ROOT/tools/small_probe.py" $P 20 > "$OUT/${TAG}pmc_sq.log" 2>&1
  step $? "${TAG}pmc sq"
  timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d "$OUT/prof/${TAG}pmc_ta" -o run --output-format csv -- python3 "$ROOT/tools/small_probe.py" $P 20 > "$OUT/${TAG}pmc_ta.log" 2>&1
  step $? "${TAG}pmc ta"
  fi
  ;;
c5)  # BASELINE configs[4]: rocprofv3 kernel trace of the full 50M x 32 x 1000 bf16 job + PMC passes on 12M items
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof/c5_job" -o run --output-format csv -- python3 "$ROOT/tools/bench_c5.py" > "$OUT/c5_job.json" 2> "$OUT/c5_job.err"
  step $? "c5 job trace"
  A="--items 12000000"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/c5_fetch" -o run --output-format csv -- python3 "$ROOT/tools/bench_c5.py" $A > "$OUT/c5_fetch.log" 2>&1
  step $? "c5 fetch"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/c5_write" -o run --output-format csv -- python3 "$ROOT/tools/bench_c5.py" $A > "$OUT/c5_write.log" 2>&1
  step $? "c5 write"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/prof/c5_sq" -o run --output-format csv -- python3 "$ROOT/tools/bench_c5.py" $A > "$OUT/c5_sq.log" 2>&1
  step $? "c5 sq"
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d "$OUT/prof/c5_lds" -o run --output-format csv -- python3 "$ROOT/tools/bench_c5.py" $A > "$OUT/c5_lds.log" 2>&1
  step $? "c5 lds"
  ;;
c5ab)  # A/B of library builds on the C5 job at 12M items (ABLIBS="base x ...", ITEMS=, REPS=), builds alternating
  for rep in $(seq 1 ${REPS:-3}); do
    for lib in ${ABLIBS:-base}; do
      if [ "$lib" = base ]; then L=$ROOT/consensus-entropy_amd/ce_amd/libce_amd.so; else L=$ROOT/tools/_diag/libce_amd_$lib.so; fi
      CE_AMD_LIB=$L timeout -k 10 200 python3 tools/bench_c5.py --items ${ITEMS:-12000000} > "$OUT/c5ab_${lib}_$rep.json" 2> "$OUT/c5ab_${lib}_$rep.err"
      step $? "c5ab $lib $rep"
    done
  done
  ;;
smallab)  # A/B of library builds on the small-pool configs: kernel traces, builds alternating (LIBS="base reg ...")
  cd /tmp
  for rep in 1 2; do
    for lib in ${LIBS:-base}; do
      if [ "$lib" = base ]; then L=$ROOT/consensus-entropy_amd/ce_amd/libce_amd.so; else L=$ROOT/tools/_diag/libce_amd_$lib.so; fi
      for c in ${CFGS:-c1 c2hc c2mix c3 c3r}; do
        CE_AMD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof/ab_${lib}_${c}_$rep" -o run --output-format csv -- python3 "$ROOT/tools/small_probe.py" $c 200 > "$OUT/ab_${lib}_${c}_$rep.log" 2>&1
        step $? "ab $lib $c $rep"
      done
    done
  done
  ;;
debug)  # the whole GPU suite once on the debug build (device bounds checks: make -C consensus-entropy_amd debug)
  CE_AMD_LIB=$ROOT/tools/_diag/libce_amd_debug.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu_debug.log" 2>&1
  step $? "pytest debug build"
  ;;
phase)  # per-block phase stamps of the C3 selection (tools/phase_probe.py) on the diagnostic build (make phase)
  for lib in ${PLIBS:-ce_amd_phase}; do  # phase-stamp builds in tools/_diag (make phase / make variant DEFS=-DCE_PHASE_TIMING ...)
    for c in ${CFGS:-c3 c1}; do
      CE_AMD_LIB=$ROOT/tools/_diag/$lib.so timeout -k 10 120 python3 tools/phase_probe.py $c > "$OUT/phase_${lib}_$c.json" 2> "$OUT/phase_${lib}_$c.err"
      step $? "phase probe $lib $c"
    done
  done
  ;;
scale)  # single-GPU proxies of one rank at 1/2/4/8 GPUs + the world-1 RCCL step, eager vs HIP graph (tools/scale_proxy.py)
  timeout -k 10 300 python3 tools/scale_proxy.py > "$OUT/scale_proxy.json" 2> "$OUT/scale_proxy.err"
  step $? "scale proxy"
  ;;
tests)  # selected GPU tests only: TESTS="file::name ..." or PYTEST_ARGS="-k expr" (failures keep going)
  timeout -k 10 ${TLIM:-600} python -u -m pytest ${TESTS:-tests} -m gpu -v -s --timeout 400 --timeout-method thread ${TESTK:+-k "$TESTK"} ${PYTEST_ARGS} > "$OUT/pytest_sel${TAG}.log" 2>&1
  step $? "pytest selected"
  ;;
gather)  # SURVEY §8(f)1 shuffled frames: the random-row probe + FETCH / WRITE passes of the fused shuffled kernel
  timeout -k 10 300 python3 tools/gather_probe.py > "$OUT/gather_probe.json" 2> "$OUT/gather_probe.err"
  step $? "gather probe"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/gather_fetch" -o run --output-format csv -- python3 "$ROOT/tools/gather_probe.py" --pmc > "$OUT/gather_fetch.log" 2>&1
  step $? "gather fetch"
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof/gather_write" -o run --output-format csv -- python3 "$ROOT/tools/gather_probe.py" --pmc > "$OUT/gather_write.log" 2>&1
  step $? "gather write"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof/gather_trace" -o run --output-format csv -- python3 "$ROOT/tools/gather_probe.py" --pmc > "$OUT/gather_trace.log" 2>&1
  step $? "gather trace"
  [ -x "$ROOT/tools/_diag/random_row_probe" ] || { echo "build it first: make -C consensus-entropy_amd probes" >> "$LOG"; exit 2; }
  timeout -k 10 120 "$ROOT/tools/_diag/random_row_probe" > "$OUT/random_rows.json" 2> "$OUT/random_rows.err"
  step $? "random row probe"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof/rows32_fetch" -o run --output-format csv -- "$ROOT/tools/_diag/random_row_probe" 32 > "$OUT/rows32_fetch.log" 2>&1
  step $? "random rows 32 fetch"
  ;;
framesab)  # the frames probe (tools/gather_probe.py) per library build (LIBS="base x"), alternating, 2 rounds
  for rep in 1 2; do
    for lib in ${LIBS:-base}; do
      if [ "$lib" = base ]; then L=$ROOT/consensus-entropy_amd/ce_amd/libce_amd.so; else L=$ROOT/tools/_diag/libce_amd_$lib.so; fi
      CE_AMD_LIB=$L timeout -k 10 200 python3 tools/gather_probe.py ${FRAMES_ARGS} > "$OUT/framesab${TAG}_${lib}_$rep.json" 2> "$OUT/framesab${TAG}_${lib}_$rep.err"
      step $? "framesab $lib $rep"
    done
  done
  ;;
memab)  # member-inference configs (bench_configs.py --only ${ONLY:-6}: 6 GNB, SGD; 7 XGB) per library build (LIBS="base x"), alternating, 2 rounds
  for rep in 1 2; do
    for lib in ${LIBS:-base}; do
      if [ "$lib" = base ]; then L=$ROOT/consensus-entropy_amd/ce_amd/libce_amd.so; else L=$ROOT/tools/_diag/libce_amd_$lib.so; fi
      CE_AMD_LIB=$L timeout -k 10 200 python3 tools/bench_configs.py --only ${ONLY:-6} > "$OUT/memab_${lib}_$rep.log" 2>&1
      step $? "memab $lib $rep"
    done
  done
  ;;
c3drain)  # the configs[2] load floor (tools/c3_drain_probe.hip: reads only, no selection) under rocprofv3
  [ -x "$ROOT/tools/_diag/c3_drain_probe" ] || { echo "build it first: make -C consensus-entropy_amd probes" >> "$LOG"; exit 2; }
  cd /tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof/${TAG}c3drain" -o run --output-format csv -- "$ROOT/tools/_diag/c3_drain_probe" 200 > "$OUT/${TAG}c3drain.json" 2> "$OUT/${TAG}c3drain.err"
  step $? "c3 drain probe"
  ;;
c5probe)  # tools/c5_probe.py per library build (LIBS="base x"), alternating, REPS rounds (prefilter-friendly and rising pools)
  for rep in $(seq 1 ${REPS:-2}); do
    for lib in ${LIBS:-base}; do
      if [ "$lib" = base ]; then L=$ROOT/consensus-entropy_amd/ce_amd/libce_amd.so; else L=$ROOT/tools/_diag/libce_amd_$lib.so; fi
      CE_AMD_LIB=$L timeout -k 10 300 python3 tools/c5_probe.py ${C5_ARGS} > "$OUT/c5probe${TAG}_${lib}_$rep.json" 2> "$OUT/c5probe${TAG}_${lib}_$rep.err"
      step $? "c5probe $lib $rep"
    done
  done
  ;;
firstcall)  # first-call latency per library build (tools/first_call.py)
  timeout -k 10 300 python3 tools/first_call.py ${LIBS} > "$OUT/first_call.json" 2> "$OUT/first_call.err"
  step $? "first call"
  ;;
*) echo "PHASE must be check, ab, profile, benchprof, configs, xgb, mpmc, small, c5, c5ab, smallab, debug, phase, firstcall, scale, gather, framesab, memab, c5probe, c3drain or tests" >&2; exit 2 ;;
esac
echo "done $PHASE $(date)" >> "$LOG"
