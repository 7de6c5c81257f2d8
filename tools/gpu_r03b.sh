#!/bin/bash
# Round-3 visit b: GPU tests, bench A/B (fold on/off, member-major DMA on/off),
# small-pool traces (tile-size variants, the r02 library), C3 PMC, first call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
b() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  echo "bench $n ok" >> $OUT/steps.log
}
b nmc python bench.py --no-cpu-baseline
b nmc_nofold CE_AMD_FOLD=0 python bench.py --no-cpu-baseline
b mnc python bench.py --no-cpu-baseline --layout MNC
b mnc_direct CE_AMD_MNC_DMA=0 python bench.py --no-cpu-baseline --layout MNC
PHASE=small bash tools/gpu_round.sh || exit $?
TAG=s4_ CFGS="c3" PMCCFG=none CE_AMD_TILE_USER=512 PHASE=small bash tools/gpu_round.sh
TAG=p512_ CFGS="c1 c2hc" CE_AMD_TILE_POOL=512 PHASE=small bash tools/gpu_round.sh
TAG=p1024_ CFGS="c1 c2hc" CE_AMD_TILE_POOL=1024 PHASE=small bash tools/gpu_round.sh
TAG=r02_ CE_AMD_LIB=$PWD/tools/_diag/libce_amd_r02.so PHASE=small bash tools/gpu_round.sh
PHASE=firstcall LIBS="tools/_diag/libce_amd_r02.so consensus-entropy_amd/ce_amd/libce_amd.so" bash tools/gpu_round.sh
