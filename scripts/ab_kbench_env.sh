#!/bin/bash
# Interleaved kernel timing of package trees ab/<name>/qfedx_amd; a variant named *_tNN runs with
# QFEDX_HEA_TILE=NN (MFMA engine tile bits).  Usage: gpurun -- 'bash scripts/ab_kbench_env.sh [kbench args]'
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
variants=$(ls -d ab/*/ | xargs -n1 basename)
for r in 1 2; do for v in $variants; do
  tb=""; case $v in *t13) tb=13;; *t14) tb=14;; esac
  QFEDX_HEA_TILE=${tb:-14} QFX_PKG_ROOT=$PWD/ab/$v timeout -k 10 200 python scripts/hea_kbench.py --iters 30 "$@" > gpurun_out/ab_$v$r.log 2>&1 || exit 1
  echo "$v$r $(tail -1 gpurun_out/ab_$v$r.log)"
done; done
