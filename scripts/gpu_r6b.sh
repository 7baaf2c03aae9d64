#!/bin/bash
# A/B of the pair-back variants (ab/*), then the 1-client (BASELINE config 2 per-GPU point) tile sweep on the base tree.
source "$(dirname "$0")/gpu_step.sh"
bash "$(dirname "$0")/gpu_ab.sh" || exit $?
for tl in "14 13" "13 13" "12 12" "12 11"; do
  set -- $tl
  TAILN=1 QFX_PKG_ROOT=$PWD/ab/base QFEDX_HEA_TILE=$1 QFEDX_HEA_ADJ_TILE=$2 step c1_t$1_$2 200 \
    python scripts/hea_kbench.py --clients 1 --iters 200
done
