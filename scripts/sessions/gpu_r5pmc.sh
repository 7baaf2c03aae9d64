#!/bin/bash
# Round 5 final: PMC counters of the MFMA statevector pass kernels (16q x 3L x 2048 samples, scripts/hea_kbench.py):
# two SQ sets, then FETCH_SIZE and WRITE_SIZE in passes of their own (TCC counter limit); kernel-trace only.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5pmc
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/r5pmc -o set$i -- python3 scripts/hea_kbench.py --iters 2 > gpurun_out/r5pmc_set$i.log 2>&1
  rc=$?; echo "set$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3 4; do python3 scripts/pmc_summary.py gpurun_out/r5pmc/set${i}_counter_collection.csv | grep -E "hea_(adj|fwd)"; done > gpurun_out/r5pmc/summary.txt; cut -c1-400 gpurun_out/r5pmc/summary.txt
