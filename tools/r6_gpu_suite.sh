set -o pipefail
mkdir -p gpurun_out/r6_suite
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail 15 -p no:cacheprovider > gpurun_out/r6_suite/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r6_suite/gpu_tests.log
exit $rc
