#!/bin/bash
# Interleaved A/B of the built package trees under ab/ (scripts/hea_kbench.py per-pass timing), 3 rounds; the first
# round also checks each tree against the fp32 VALU engine (--precision).  KBENCH / KARGS select another timer.
source "$(dirname "$0")/gpu_step.sh"
variants=$(ls -d ab/*/ | xargs -n1 basename)
for r in 1 2 3; do for v in $variants; do
  extra=""; [ $r -eq 1 ] && [ -z "$KBENCH" ] && extra="--precision"
  TAILN=1 QFX_PKG_ROOT=$PWD/ab/$v step ab_${TAG}${v}$r 200 python ${KBENCH:-scripts/hea_kbench.py} --iters 30 $extra $KARGS
done; done
