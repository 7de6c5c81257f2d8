#!/bin/bash
# pytest -m gpu, then the latency probe, the per-config bench and bench.py;
# each GPU step has its own limit and a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/quick_steps.log
st() { echo "$2: $1" >> $OUT/quick_steps.log; case $1 in 0) ;; *) exit $1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
st $? pytest
[ -n "$SKIP_PROBE" ] || { timeout -k 10 200 python tools/latency_probe.py > $OUT/lat.json 2> $OUT/lat.err; st $? probe; }
[ -n "$SKIP_CONFIGS" ] || { timeout -k 10 300 python tools/bench_configs.py > $OUT/configs.json 2> $OUT/configs.err; st $? configs; }
[ -n "$SKIP_BENCH" ] || { timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; st $? bench; }
echo done >> $OUT/quick_steps.log
