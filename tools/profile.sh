#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel-trace stats, then one PMC
# pass per counter group (never combined with tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/prof; mkdir -p $OUT
export TMPDIR=/tmp
LAYOUT=${LAYOUT:-NMC}
BENCH="$ROOT/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --layout $LAYOUT ${BENCH_ARGS}"
cd /tmp
step() { local s=$1 name=$2; echo "$name: $s" >> $OUT/steps.log; case $s in 0) ;; *) exit $s ;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$LAYOUT -o run --output-format csv -- python3 $BENCH > $OUT/trace_$LAYOUT.log 2>&1
step $? trace
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$LAYOUT -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --layout $LAYOUT ${BENCH_ARGS} > $OUT/fetch_$LAYOUT.log 2>&1
step $? fetch
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$LAYOUT -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --layout $LAYOUT ${BENCH_ARGS} > $OUT/write_$LAYOUT.log 2>&1
step $? write
