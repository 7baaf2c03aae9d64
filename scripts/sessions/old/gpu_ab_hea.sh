# MFMA engine tests, then interleaved A/B kernel timing of the trees under ab/ (scripts/ab_kbench.sh)
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hea_tests.log 2>&1; rc=$?; tail -2 gpurun_out/hea_tests.log; [ $rc -eq 0 ] && bash scripts/ab_kbench.sh "$@"
