#!/bin/bash
# Round 5, call 3: chained pair ops -- MFMA-engine GPU tests first (pair vs unpaired, dense oracle), then the full GPU
# suite, the headline + 8-client bench, pair A/B (QFEDX_HEA_PAIR) interleaved, stall attribution.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5c/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5c/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
step hea_tests 400 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench64 300 python bench.py --steps 20 --warmup 3
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step ab_pair64 300 python -u scripts/hea_ab.py --rounds 7 --variants "single:env.QFEDX_HEA_PAIR=0,pair:env.QFEDX_HEA_PAIR=7"
step ab_pair8 300 python -u scripts/hea_ab.py --rounds 7 --clients 8 --iters 30 --variants "single:env.QFEDX_HEA_PAIR=0,pair:env.QFEDX_HEA_PAIR=7"
step stamps64 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5c/stamps64.jsonl
step prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5c/prof -o bench -- python3 bench.py --steps 10 --warmup 3
step cnn_kbench 150 python3 scripts/cnn_kbench.py
step cnn_pmc_b 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES --output-format csv -d gpurun_out/r5c/pmcc -o setb -- python3 scripts/cnn_kbench.py --iters 2
python3 scripts/pmc_summary.py gpurun_out/r5c/pmcc/setb_counter_collection.csv > gpurun_out/r5c/cnn_pmc_b.txt 2>&1
step cfed 300 python3 bench_suite.py --config cfed128 --steps 10 --warmup 3
