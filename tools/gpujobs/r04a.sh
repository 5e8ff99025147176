set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py "tests/test_gpu_jpeg.py::test_file_caller_stage_fused_cases" -x -v --timeout 180 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r04a_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config plan --steps 3 --warmup 1 > gpurun_out/r04a_plan.json 2> gpurun_out/r04a_plan.err
rc=$?
cat gpurun_out/r04a_plan.json; tail -5 gpurun_out/r04a_plan.err
exit $rc
