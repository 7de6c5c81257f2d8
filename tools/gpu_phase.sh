#!/bin/bash
# per-block phase stamps of the C3 selection (tools/phase_probe.py) per diagnostic library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for v in ${LIBS:-libce_amd_ph}; do
  CE_AMD_LIB=$PWD/tools/_diag/$v.so timeout -k 10 120 python tools/phase_probe.py > $OUT/phase_$v.json 2> $OUT/phase_$v.err || exit $?
  echo "phase $v ok" >> $OUT/steps.log
done
