#!/bin/bash
# Round 4, call 7: CFed conv-kernel PMC + round timeline, SecAgg full vs sparse suite lines, and the RCCL A/B at the
# 8-client share (one-rank RCCL process group vs none).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profc
bash scripts/gpu_cnn_pmc.sh > gpurun_out/r4g_cnn_pmc.txt 2>&1 || { tail -5 gpurun_out/r4g_cnn_pmc.txt; exit 1; }
cat gpurun_out/r4g_cnn_pmc.txt | cut -c1-400
STEPS=10 WARMUP=3 bash scripts/gpu_suite.sh cfed128 cfed128_secagg cfed128_secagg_sparse vqc16q_64_mfma_secagg_sparse || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profc -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3 > gpurun_out/r4g_cfed_prof.log 2>&1 || { tail -5 gpurun_out/r4g_cfed_prof.log; exit 1; }
python3 scripts/round_timeline.py gpurun_out/profc/cfed_kernel_trace.csv | tee gpurun_out/r4g_cfed_timeline.txt
for be in none nccl; do
  if [ $be = none ]; then
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --clients 8 > gpurun_out/r4g_share8_$be.log 2>&1 || { tail -5 gpurun_out/r4g_share8_$be.log; exit 1; }
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 40 --warmup 5 --clients 8 --dist-backend nccl > gpurun_out/r4g_share8_$be.log 2>&1 || { tail -5 gpurun_out/r4g_share8_$be.log; exit 1; }
  fi
  grep '"metric"' gpurun_out/r4g_share8_$be.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$be', r['ms_per_step'], r.get('graph_comm'), r.get('rccl_world_size'), r.get('dist_backend'))"
done
