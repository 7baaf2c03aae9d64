cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hea14.log 2>&1; rc=$?; tail -2 gpurun_out/hea14.log; [ $rc -eq 0 ] || exit $rc
QFEDX_HEA_TILE=13 timeout -k 10 300 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hea13.log 2>&1; rc=$?; tail -2 gpurun_out/hea13.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_kbench_env.sh
