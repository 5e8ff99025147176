set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_jpeg.py -k "plan or stage or truncated or corrupted" -q --timeout 180 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04e_tests.log
bash tools/profile_bench.sh r04e_plan --config plan --steps 3 --warmup 1 --plan-no-loop || exit 1
head -12 gpurun_out/prof_r04e_plan/kstats.txt
bash tools/profile_bench.sh r04e_jpeg --config jpeg --steps 3 --warmup 1 || exit 1
head -10 gpurun_out/prof_r04e_jpeg/kstats.txt
timeout -k 10 300 python -u bench.py --config plan --steps 3 --warmup 1 > gpurun_out/r04e_plan.json 2> gpurun_out/r04e_plan.err || exit 1
cat gpurun_out/r04e_plan.json
exit $rc
