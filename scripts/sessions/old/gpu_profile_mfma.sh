#!/bin/bash
# MFMA-engine evidence: headline bench, suite configs (VALU vs MFMA), rocprofv3 kernel stats, PMC counters.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profm gpurun_out/pmcm
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" || tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step bench_mfma 600 python bench.py --steps 20 --warmup 3
step bench_valu 600 python bench.py --steps 20 --warmup 3 --engine valu
step suite_20q_valu 600 python bench_suite.py --config vqc20q_dp64 --steps 10 --warmup 2
step suite_20q_mfma 600 python bench_suite.py --config vqc20q_dp64_mfma --steps 10 --warmup 2
step prof_mfma 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profm -o bench -- python3 bench.py --steps 10 --warmup 2
step pmc_mfma1 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmcm -o set1 -- python3 scripts/hea_kbench.py --iters 2
step pmc_mfma2 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcm -o set2 -- python3 scripts/hea_kbench.py --iters 2
# FETCH_SIZE takes 3 of the 4 TCC counters and WRITE_SIZE 2: one pass each
step pmc_mfma3 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcm -o set3 -- python3 scripts/hea_kbench.py --iters 2
step pmc_mfma4 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcm -o set4 -- python3 scripts/hea_kbench.py --iters 2
