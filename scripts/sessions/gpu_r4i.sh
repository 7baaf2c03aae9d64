#!/bin/bash
# Round 4, call 9: fused readout with the partials prefetched across the last wave's lanes: HEA GPU tests, A/B of the
# local step (fused vs separate readout kernel) at 64 and 8 clients, share-8 timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof6
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_hea.py tests/test_gpu_kernels.py > gpurun_out/r4i_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4i_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/hea_ab.py --rounds 7 --variants "sep:env.QFEDX_FUSED_READOUT=0,fused:env.QFEDX_FUSED_READOUT=1" > gpurun_out/r4i_ab64.log 2>&1 || { tail -5 gpurun_out/r4i_ab64.log; exit 1; }
tail -1 gpurun_out/r4i_ab64.log
timeout -k 10 300 python -u scripts/hea_ab.py --rounds 7 --clients 8 --iters 30 --variants "sep:env.QFEDX_FUSED_READOUT=0,fused:env.QFEDX_FUSED_READOUT=1" > gpurun_out/r4i_ab8.log 2>&1 || { tail -5 gpurun_out/r4i_ab8.log; exit 1; }
tail -1 gpurun_out/r4i_ab8.log
for v in 0 1; do
  QFEDX_FUSED_READOUT=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 --clients 8 > gpurun_out/r4i_share8_$v.log 2>&1 || exit 1
  echo "fused=$v $(grep '"metric"' gpurun_out/r4i_share8_$v.log | cut -c150-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8 > gpurun_out/r4i_prof8.log 2>&1 || exit 1
python3 scripts/round_timeline.py gpurun_out/prof6/share8_kernel_trace.csv | tee gpurun_out/r4i_share8_timeline.txt
