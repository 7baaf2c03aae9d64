#!/bin/bash
# MALL residency probe: per-step time of the 16q x 3L MFMA step vs client count (32 samples each), plain vs
# non-temporal tile stores.  If a pass's states that fit the 256 MB Infinity Cache run super-linearly faster, client
# chunks sized to it beat one 64-client pass sequence.
source "$(dirname "$0")/gpu_step.sh"
for r in 1 2; do for c in 16 24 32 40 48 64; do for nt in 0 1; do
  TAILN=1 QFEDX_HEA_NT=$nt step mall_c${c}_nt${nt}_$r 200 python scripts/hea_kbench.py --clients $c --iters 40
done; done; done
