#!/bin/bash
# Round 5, call 20: PMC (issue / wait counters) of the CFed round's kernels (bench_suite cfed128, a few rounds).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/r5t -o seta -- python3 bench_suite.py --config cfed128 --steps 2 --warmup 1 > gpurun_out/r5t/seta.log 2>&1
rc=$?; echo "seta rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/r5t/seta_counter_collection.csv > gpurun_out/r5t/seta_summary.txt 2>&1
cat gpurun_out/r5t/seta_summary.txt | cut -c1-400
