#!/bin/bash
# Round 4, call 14: headline A/B of the merged round start (QFEDX_ROUND_START) and the fused single-rank apply
# (QFEDX_FUSED_APPLY), interleaved, plus a kernel trace of the headline with both on and both off.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof9
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*'
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
  QFEDX_ROUND_START=0 QFEDX_FUSED_APPLY=0 step r4n_h_00_$rep 200 python bench.py --steps 40 --warmup 5
  QFEDX_ROUND_START=1 QFEDX_FUSED_APPLY=0 step r4n_h_10_$rep 200 python bench.py --steps 40 --warmup 5
  QFEDX_ROUND_START=0 QFEDX_FUSED_APPLY=1 step r4n_h_01_$rep 200 python bench.py --steps 40 --warmup 5
  QFEDX_ROUND_START=1 QFEDX_FUSED_APPLY=1 step r4n_h_11_$rep 200 python bench.py --steps 40 --warmup 5
done
QFEDX_ROUND_START=1 QFEDX_FUSED_APPLY=1 step r4n_prof_on 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o on -- python3 bench.py --steps 10 --warmup 3
QFEDX_ROUND_START=0 QFEDX_FUSED_APPLY=0 step r4n_prof_off 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o off -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof9/on_kernel_trace.csv --marker qfx_fedavg_reduce_kernel
python3 scripts/round_timeline.py gpurun_out/prof9/off_kernel_trace.csv --marker qfx_fedavg_reduce_kernel
