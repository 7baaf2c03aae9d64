#!/bin/bash
# Round 4, call 6: headline + 8-client share benches, kernel-trace round timelines, and the four PMC counter sets of the
# MFMA pass kernels (16q x 3L x 2048 samples) after the epilogue change.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof4 gpurun_out/pmc4
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | cut -c1-330
  [ $rc -eq 0 ] || exit $rc
}
step r4f_bench64 300 python bench.py --steps 20 --warmup 5
step r4f_share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step r4f_prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof4 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8
step r4f_prof64 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof4 -o full64 -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof4/share8_kernel_trace.csv > gpurun_out/r4f_share8_timeline.txt
python3 scripts/round_timeline.py gpurun_out/prof4/full64_kernel_trace.csv > gpurun_out/r4f_full64_timeline.txt
cat gpurun_out/r4f_share8_timeline.txt gpurun_out/r4f_full64_timeline.txt
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc4 -o set$i -- python3 scripts/hea_kbench.py --iters 2 > gpurun_out/pmc4_set$i.log 2>&1
  rc=$?; echo "set$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3 4; do python3 scripts/pmc_summary.py gpurun_out/pmc4/set${i}_counter_collection.csv | grep -E "hea_(adj|fwd)" > gpurun_out/r4f_pmc_set$i.txt; cat gpurun_out/r4f_pmc_set$i.txt | cut -c1-400; done
