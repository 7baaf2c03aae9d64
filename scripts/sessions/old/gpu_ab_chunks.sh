#!/bin/bash
# A/B of client chunks per MFMA training step (QFEDX_HEA_CHUNKS, staggered streams): the bitwise test, then
# interleaved bench.py runs of the headline (64 clients) and the 8-client per-rank share on one box.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hea.py -k chunked -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/chunk_test.log 2>&1
rc=$?; tail -3 gpurun_out/chunk_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for n in ${CHUNKS:-1 2 3 4}; do
    for cl in 64 8; do
      QFEDX_HEA_CHUNKS=$n timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 5 --clients $cl \
        > gpurun_out/abc_${n}_${cl}_$r.log 2>&1 || exit 1
      echo "chunks=$n clients=$cl r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abc_${n}_${cl}_$r.log)"
    done
  done
done
