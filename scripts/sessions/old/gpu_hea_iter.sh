#!/bin/bash
# MFMA engine iteration: numerics tests -> per-phase ablation -> kernel timing -> headline bench (stop at first failure)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step hea_tests 600 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAILN=30 step ablate 300 python3 scripts/hea_ablate.py
TAILN=2 step hea_kbench 300 python scripts/hea_kbench.py
TAILN=2 step bench 600 python bench.py --steps 20 --warmup 3
exit 0
