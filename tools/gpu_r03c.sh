#!/bin/bash
# Round-3 visit c: GPU tests; bench fold A/B; small-pool traces (single-block
# defaults); C5 wide-stream A/B libraries; fast-division check; scaling proxies.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash tools/gpu_tests_then.sh || exit $?
b() {  # name, env/cmd...
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || exit $?
  echo "bench $n ok" >> $OUT/steps.log
}
b nmc python bench.py --no-cpu-baseline
b nmc_nofold CE_AMD_FOLD=0 python bench.py --no-cpu-baseline
b mnc python bench.py --no-cpu-baseline --layout MNC
CFGS="c1 c2hc c2mix c3 c3r" PMCCFG=none PHASE=small bash tools/gpu_round.sh || exit $?
CE_AMD_LIB=$PWD/tools/_diag/libce_amd_fastdiv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s -k "row_division or golden or large or entropy_bit" --timeout 240 --timeout-method thread > $OUT/pytest_fastdiv.log 2>&1
echo "fastdiv tests rc=$?" >> $OUT/steps.log
for L in "" wlds wlds4 fastdiv; do
  lib=""; [ -n "$L" ] && lib=CE_AMD_LIB=$PWD/tools/_diag/libce_amd_$L.so
  timeout -k 10 300 env $lib python tools/bench_c5.py --items 12000000 --chunk 2000000 > $OUT/c5_${L:-base}.json 2> $OUT/c5_${L:-base}.err || exit $?
  echo "c5 ${L:-base} ok" >> $OUT/steps.log
done
timeout -k 10 300 python tools/scale_proxy.py > $OUT/scale_proxy.json 2> $OUT/scale_proxy.err
echo "scale proxy rc=$?" >> $OUT/steps.log
