#!/bin/bash
# Round 5 final validation (second run, final tree) on one MI355X: GPU suite, smoke, headline and 8-client benches, headline round timeline,
# then every BASELINE suite line except config 5 (its 26.7 s rounds ran in call 11, profiles/r5_bench_lines_r5k.jsonl).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5final2
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5final2/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/r5final2/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench64 300 python bench.py --steps 20 --warmup 3
step bench64b 300 python bench.py --steps 20 --warmup 3
step share8 300 python bench.py --steps 40 --warmup 5 --clients 8
step share8b 300 python bench.py --steps 40 --warmup 5 --clients 8
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5final2/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5final2/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5final2/timeline64.txt 2>&1
for c in cfed128 cfed128_epoch cfed128_secagg cfed128_secagg_sparse vqc16q_64_mfma vqc16q_64_mfma_secagg \
         vqc16q_64_mfma_secagg_sparse vqc16q_bf16_8_mfma vqc16q_fp16_8_mfma vqc20q_dp64_mfma vqc20q_ddp64_mfma \
         vqc48q_mps64; do
  step suite_$c 400 python bench_suite.py --config $c --steps 10 --warmup 2
  grep '"metric"' gpurun_out/r5final2/suite_$c.log >> gpurun_out/r5final2/suite_lines.jsonl
done
