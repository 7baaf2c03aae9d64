#!/bin/bash
# Round-3 fusions (Adam in the gradient reduction, round signal in the upload kernel, scratch-free frag and
# product-state kernels): full GPU suite, smoke, headline bench, 8-client share, and the round timelines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_share8_prof.sh
