#!/bin/bash
# Adjoint pass-kernel breakdown: per-phase ablation timing + wait/issue PMC counters of the MFMA engine step.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmca
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step ablate 300 python3 scripts/hea_ablate.py
step pmc_a 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmca -o seta -- python3 scripts/hea_kbench.py --iters 2
step pmc_b 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmca -o setb -- python3 scripts/hea_kbench.py --iters 2
step pmc_c 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmca -o setc -- python3 scripts/hea_kbench.py --iters 2
