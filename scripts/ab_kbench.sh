#!/bin/bash
# A/B kernel timing of two built package trees, interleaved to cancel box drift.
# Prepare on the CPU:  mkdir -p ab/A ab/B; cp -r qfedx_amd ab/A/  (build variant B) cp -r qfedx_amd ab/B/
# then: gpurun -- 'bash scripts/ab_kbench.sh'   (delete ab/ afterwards so later calls do not ship it)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do for v in A B; do
  QFX_PKG_ROOT=$PWD/ab/$v timeout -k 10 200 python scripts/hea_kbench.py --iters 30 "$@" > gpurun_out/ab_$v$r.log 2>&1 || exit 1
  echo "$v$r $(tail -1 gpurun_out/ab_$v$r.log)"
done; done
