#!/bin/bash
# Round-3 visit q: rocprofv3 of the driver's exact bench command + FETCH/WRITE
# passes (NMC), and the member-major layout's trace + FETCH/WRITE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PHASE=benchprof bash tools/gpu_round.sh || exit $?
PHASE=profile LAYOUT=MNC bash tools/gpu_round.sh || exit $?
