#!/bin/bash
# One GPU round: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fault() {  # $1 = exit status, $2 = step name
  case "$1" in
    0|1) return 0 ;;
    *) echo "STEP $2 ended with status $1 -- stopping" | tee -a "$OUT/steps.log"; exit "$1" ;;
  esac
}
echo "start $(date)" > "$OUT/steps.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1
s=$?; echo "pytest gpu: $s" >> "$OUT/steps.log"; stop_if_fault $s pytest
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
s=$?; echo "smoke: $s" >> "$OUT/steps.log"; stop_if_fault $s smoke
timeout -k 10 400 python bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err"
s=$?; echo "bench: $s" >> "$OUT/steps.log"; stop_if_fault $s bench
if [ -z "$NO_PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1
  s=$?; echo "rocprof: $s" >> "$OUT/steps.log"; stop_if_fault $s rocprof
fi
echo "done $(date)" >> "$OUT/steps.log"
