#!/bin/bash
# Static wave priority A/B (ab/p0..p3: QFX_HEA_PRIO off / forward / adjoint / both) at 64 and 8 clients, then the CC4
# kernel trace of a one-rank RCCL bench (QFEDX_CC4=1) for scripts/cc4_overlap.py.
source "$(dirname "$0")/gpu_step.sh"
bash "$(dirname "$0")/gpu_ab.sh" || exit $?
TAG=c8_ KARGS="--clients 8 --iters 100" KBENCH=scripts/hea_kbench.py bash "$(dirname "$0")/gpu_ab.sh" || exit $?
export QFEDX_CC4=1
step prof_cc4 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cc4 -o cc4 -- \
  python3 bench.py --dist-backend nccl --clients 8 --steps 20 --warmup 3
