#!/bin/bash
# Round 6: PMC of the final tree's hot kernels - the MFMA statevector passes (scripts/gpu_pmc_hea_now.sh) and the
# split-fp16 CFed conv kernels (scripts/gpu_cnn_pmc.sh); counter sets in runs of their own, kernel-trace only.
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_pmc_hea_now.sh > gpurun_out/pmc_hea_summary.txt 2>&1 || { tail -5 gpurun_out/pmc_hea_summary.txt; exit 1; }
tail -12 gpurun_out/pmc_hea_summary.txt
bash scripts/gpu_cnn_pmc.sh > gpurun_out/pmc_cnn_summary.txt 2>&1 || { tail -5 gpurun_out/pmc_cnn_summary.txt; exit 1; }
tail -8 gpurun_out/pmc_cnn_summary.txt
