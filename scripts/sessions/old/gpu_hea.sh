#!/bin/bash
# MFMA engine: numerics tests -> kernel timing -> PMC counters of the passes -> headline bench (stop at first failure)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step hea_tests 600 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
TAILN=2 step hea_kbench 300 python scripts/hea_kbench.py
if [ -n "$PMC" ]; then
  step hea_pmc 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc -o hea -- python3 scripts/hea_kbench.py --iters 2
fi
[ -n "$BENCH" ] && step hea_bench 600 python bench.py --steps 20 --warmup 3 --engine mfma
exit 0
