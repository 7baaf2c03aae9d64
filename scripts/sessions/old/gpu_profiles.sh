#!/bin/bash
# Profile evidence: kernel stats of the headline + CFed benches, PMC counters of the VQC passes and the
# CNN kernels (kernel-trace + pmc only; no sys/runtime traces with counters).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
rocprofv3 -L > gpurun_out/profiles/avail_counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profiles -o bench16 -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/profiles/bench16.log 2>&1
echo "bench16 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profiles -o cfed -- python3 bench_suite.py --config cfed128 --steps 5 --warmup 2 > gpurun_out/profiles/cfed.log 2>&1
echo "cfed rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/profiles -o cfed_pmc1 -- python3 bench_suite.py --config cfed128 --steps 1 --warmup 1 > gpurun_out/profiles/cfed_pmc1.log 2>&1
echo "cfed_pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/profiles -o cfed_pmc2 -- python3 bench_suite.py --config cfed128 --steps 1 --warmup 1 > gpurun_out/profiles/cfed_pmc2.log 2>&1
echo "cfed_pmc2 rc=$?"
bash scripts/gpu_pmc.sh > gpurun_out/profiles/vqc_pmc.log 2>&1
echo "vqc pmc rc=$?"
exit 0
