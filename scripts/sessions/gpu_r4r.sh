#!/bin/bash
# Round 4, call 18: group-op address words staged pre-shifted (op_word): HEA GPU tests, interleaved kernel A/B
# (ab/old vs ab/new), adjoint/forward PMC set 1 of the new tree, headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc5
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_hea.py tests/test_gpu_debug_build.py > gpurun_out/r4r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4r_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_kbench.sh || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc5 -o set1 -- python3 scripts/hea_kbench.py --iters 2 > gpurun_out/pmc5_set1.log 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc5/set1_counter_collection.csv | grep -E "hea_(adj|fwd)" | cut -c1-400
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/r4r_bench$r.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4r_bench$r.log
done
