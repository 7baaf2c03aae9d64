#!/bin/bash
# Fused-Adam grad reduce with one release per block: kernel test, then the 8-client and 64-client round timelines
# with the fused Adam on and off (QFEDX_FUSED_ADAM=0).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof9
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E '"metric"|passed|failed' "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "adam or padded or upload"
for v in 1 0; do
  export QFEDX_FUSED_ADAM=$v
  step prof8_$v 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o s8_$v -- python3 bench.py --steps 20 --warmup 3 --clients 8
  step prof64_$v 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o f64_$v -- python3 bench.py --steps 10 --warmup 3
  python3 scripts/round_timeline.py gpurun_out/prof9/s8_${v}_kernel_trace.csv | head -4
  python3 scripts/round_timeline.py gpurun_out/prof9/f64_${v}_kernel_trace.csv | head -4
done
