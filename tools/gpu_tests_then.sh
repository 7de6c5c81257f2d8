#!/bin/bash
# pytest -m gpu first; only if it passes (or merely has failing tests: rc 1)
# run the rest of the command line.  A GPU fault, abort or time-out (any
# other rc) stops the call here.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/steps.log
tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
if [ $# -gt 0 ]; then bash -c "$*"; exit $?; fi
exit $rc
