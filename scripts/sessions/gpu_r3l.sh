#!/bin/bash
# Session re-entry validation (full GPU suite, smoke, headline bench + kernel stats) followed by the
# gate-precision A/B: ab/base (fp16 hi + lo gate halves) vs ab/nolo (-DQFX_HEA_GATE_LO=0), interleaved, with
# errors against the fp32 VALU engine.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
for r in 1 2; do for v in base nolo; do
  QFX_PKG_ROOT=$PWD/ab/$v timeout -k 10 200 python scripts/hea_kbench.py --iters 30 --precision > gpurun_out/ab_$v$r.log 2>&1 || exit 1
  echo "$v$r $(tail -1 gpurun_out/ab_$v$r.log)"
done; done
