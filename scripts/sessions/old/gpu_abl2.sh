#!/bin/bash
# Adjoint-kernel time decomposition (ablation build ab/abl, scripts/hea_kbench.py): bits 1 barriers, 2 grad
# atomics, 4 cross, 8 apply, 16 region flush, 32 tile load, 64 record/fragment staging.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do
  for m in 0 12 14 15 30 46 78 110 126 127; do
    QFEDX_HEA_ABLATE=$m QFX_PKG_ROOT=$PWD/ab/abl timeout -k 10 200 python scripts/hea_kbench.py --iters 20 --clients 64 > gpurun_out/abl2_${m}_$r.log 2>&1 || exit 1
    echo "abl=$m r$r $(tail -1 gpurun_out/abl2_${m}_$r.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["adj0"]["ms"], d["adj1"]["ms"], d["step_ms"])')"
  done
done
