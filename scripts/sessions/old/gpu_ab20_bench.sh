cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/ab_kbench.sh --qubits 20 --layers 2 --clients 32 --batch 16 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; grep metric gpurun_out/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --clients 8 > gpurun_out/share8.log 2>&1; rc=$?; grep metric gpurun_out/share8.log | cut -c1-200; exit $rc
