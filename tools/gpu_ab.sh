#!/bin/bash
# A/B of stage-1 variants on the bench workload; each run has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
run() { # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/ab_$name.json 2> $OUT/ab_$name.err
  local s=$?; echo "$name: $s" >> $OUT/ab_steps.log
  case $s in 0|1) ;; *) exit $s ;; esac
}
: > $OUT/ab_steps.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
s=$?; echo "pytest: $s" >> $OUT/ab_steps.log; case $s in 0|1) ;; *) exit $s ;; esac
run nmc_stream  CE_AMD_STREAM=1 python bench.py --no-cpu-baseline --steps 10 --layout NMC
run mnc_stream  CE_AMD_STREAM=1 python bench.py --no-cpu-baseline --steps 10 --layout MNC
run nmc_block   CE_AMD_STREAM=0 python bench.py --no-cpu-baseline --steps 10 --layout NMC
run mnc_block   CE_AMD_STREAM=0 python bench.py --no-cpu-baseline --steps 10 --layout MNC
