# The JPEG pass-variant tests in child processes (incl. the plain-stream reader).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 240 --timeout-method thread -k "write_and_sync_variants" > gpurun_out/r04al_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04al_tests.log
exit $rc
