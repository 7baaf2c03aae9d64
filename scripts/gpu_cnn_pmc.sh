#!/bin/bash
# CFed conv kernels alone: timing + issue/wait and LDS PMC counters (one counter set per run).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step cnn_kbench 120 python3 scripts/cnn_kbench.py
step cnn_pmc_a 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmcc -o seta -- python3 scripts/cnn_kbench.py --iters 2
step cnn_pmc_b 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES --output-format csv -d gpurun_out/pmcc -o setb -- python3 scripts/cnn_kbench.py --iters 2
for f in gpurun_out/pmcc/seta_counter_collection.csv gpurun_out/pmcc/setb_counter_collection.csv; do python3 scripts/pmc_summary.py $f | grep cnn_; done
