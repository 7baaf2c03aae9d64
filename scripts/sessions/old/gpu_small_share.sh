#!/bin/bash
# per-rank share of the strong-scaling bench: 64/N clients on one GPU (N = 8, 4, 2) + kernel trace at N=8
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_small
for c in 8 16 32; do
  timeout -k 10 300 python bench.py --clients $c --steps 30 --warmup 3 > gpurun_out/small_$c.log 2>&1
  rc=$?; echo "clients=$c rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/small_$c.log)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_small -o small -- python3 bench.py --clients 8 --steps 20 --warmup 3 > gpurun_out/prof_small.log 2>&1
echo "prof rc=$?"
