#!/bin/bash
# Round 5, call 7: chained pass launches (hea_chain, fence-free sc1 hand-off) - bitwise test vs per-pass launches first, then chain A/B at 64 and
# 8 clients (interleaved, QFEDX_HEA_CHAIN), headline + 8-client bench, kernel traces of both (dispatch counts).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5g
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5g/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5g/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
step chain_test 300 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "chained or pair or fused_readout or graph"
step hea_tests 400 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step ab_chain64 300 python -u scripts/hea_ab.py --rounds 7 --variants "single:env.QFEDX_HEA_CHAIN=0,chain:env.QFEDX_HEA_CHAIN=1"
step ab_chain8 300 python -u scripts/hea_ab.py --rounds 7 --clients 8 --iters 30 --variants "single:env.QFEDX_HEA_CHAIN=0,chain:env.QFEDX_HEA_CHAIN=1"
step ab_ro64 300 python -u scripts/hea_ab.py --rounds 7 --variants "sep:env.QFEDX_FUSED_READOUT=0,fused:env.QFEDX_FUSED_READOUT=1"
step ab_ro8 300 python -u scripts/hea_ab.py --rounds 7 --clients 8 --iters 30 --variants "sep:env.QFEDX_FUSED_READOUT=0,fused:env.QFEDX_FUSED_READOUT=1"
step stamps64 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5g/stamps64.jsonl
step bench64 300 python bench.py --steps 20 --warmup 3
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
step prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g/prof8 -o bench -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/r5g/prof64/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5g/timeline64.txt 2>&1
python3 scripts/round_timeline.py gpurun_out/r5g/prof8/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5g/timeline8.txt 2>&1
cat gpurun_out/r5g/timeline64.txt gpurun_out/r5g/timeline8.txt
