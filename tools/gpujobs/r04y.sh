set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plan.py tests/test_gpu_resize.py -q -x --timeout 180 --timeout-method thread -k "stage or plan or icon or resize" > gpurun_out/r04y_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04y_tests.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_r04y_plan
bash tools/profile_bench.sh r04y_plan --config plan --steps 4 --warmup 1 --plan-no-loop > /dev/null || exit 1
grep "resize_desc\|plan_rows\|haar_multi" gpurun_out/prof_r04y_plan/kstats.txt
timeout -k 10 600 python -u bench.py --config plan > gpurun_out/r04y_bench_plan.json 2> gpurun_out/r04y_bench_plan.err || exit 1
grep -o '"value": [0-9.]*' gpurun_out/r04y_bench_plan.json
