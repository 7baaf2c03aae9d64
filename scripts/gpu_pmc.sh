#!/bin/bash
# PMC counter collection for the statevector passes (kernel-trace only, no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 python3 scripts/kbench.py "$@" > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep step_ms gpurun_out/kbench.log
[ $rc -eq 0 ] || exit $rc
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
           "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc -o set$i -- python3 scripts/kbench.py --iters 1 "$@" > gpurun_out/pmc_set$i.log 2>&1
  rc=$?; echo "set$i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
