#!/bin/bash
# Round 6: param-shift branch dispatch (in_rep rows of one stored tile on one XCD) and the generic MPS kernel -
# tests, the non-chain MPS step timing, then the interleaved param-shift A/B.
source "$(dirname "$0")/gpu_step.sh"
step ps_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_paramshift.py
step mpo_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mps.py
step mpo_bench 300 python scripts/mps_generic_bench.py
KBENCH=scripts/ps_kbench.py KARGS="--clients 16 --batch 8 --iters 2" TAG=ps bash scripts/gpu_ab.sh
