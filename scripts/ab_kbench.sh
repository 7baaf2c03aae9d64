#!/bin/bash
# Interleaved kernel timing of several built package trees (cancels box drift between variants).
# Prepare on the CPU: one directory per variant, ab/<name>/qfedx_amd (a copy of the built package), then
#   gpurun -- 'bash scripts/ab_kbench.sh [kbench args]'
# and delete ab/ afterwards so later calls do not ship it.  KBENCH=scripts/cnn_kbench.py selects another timer.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
variants=$(ls -d ab/*/ | xargs -n1 basename)
for r in 1 2; do for v in $variants; do
  QFX_PKG_ROOT=$PWD/ab/$v timeout -k 10 200 python ${KBENCH:-scripts/hea_kbench.py} --iters 30 "$@" > gpurun_out/ab_$v$r.log 2>&1 || exit 1
  echo "$v$r $(tail -1 gpurun_out/ab_$v$r.log)"
done; done
