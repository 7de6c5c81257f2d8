#!/bin/bash
# Round-3 visit i: GPU tests, C3 phase stamps, small-pool traces (leaner survivor append / ranking)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
bash tools/gpu_phase.sh || exit $?
TAG=${TAG:-i_} CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
