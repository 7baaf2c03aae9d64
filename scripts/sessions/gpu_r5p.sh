#!/bin/bash
# Round 5, call 16: the forward pass's layer-1 inputs requested first (prefetch) vs after the record / fragment
# requests - interleaved kernel timing of two built trees (ab/base, ab/pre) at 64 and 8 clients.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
for c in 64 8; do
  for r in 1 2 3; do for v in base pre; do
    QFX_PKG_ROOT=$PWD/ab/$v timeout -k 10 200 python scripts/hea_kbench.py --iters 30 --clients $c > gpurun_out/r5p/ab_${v}_${c}_$r.log 2>&1 || exit 1
    echo "$v c=$c r=$r $(tail -1 gpurun_out/r5p/ab_${v}_${c}_$r.log)"
  done; done
done
