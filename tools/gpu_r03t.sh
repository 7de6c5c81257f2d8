#!/bin/bash
# Round-3 visit t: GPU suite + small traces on the new defaults (f64 pools UNR 4, one-member tables UNR 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_tests_then.sh || exit $?
TAG=t_ CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
