#!/bin/bash
# Round 6: pair-symmetric SecAgg mask kernel - GPU tests, then the cfed128_secagg suite line A/B (per-client vs
# pair-symmetric mask generation) and a kernel-stats profile of the new path.
source "$(dirname "$0")/gpu_step.sh"
step t_sa 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k secagg
for i in 1 2; do
  TAILN=1 step sa_old$i 300 env QFEDX_SECAGG_PAIRSYM=0 python bench_suite.py --config cfed128_secagg --steps 10 --warmup 2
  TAILN=1 step sa_new$i 300 env QFEDX_SECAGG_PAIRSYM=1 python bench_suite.py --config cfed128_secagg --steps 10 --warmup 2
done
step prof_sa 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sa2 -o sa -- python3 bench_suite.py --config cfed128_secagg --steps 5 --warmup 2
