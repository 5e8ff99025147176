set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04aa_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04aa_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
WICCA_JPEG_TIMING=1 timeout -k 10 600 python -u bench.py --config plan > gpurun_out/r04aa_bench_plan_$i.json 2> gpurun_out/r04aa_bench_plan_$i.err || exit 1
grep -o '"value": [0-9.]*' gpurun_out/r04aa_bench_plan_$i.json; grep "wicca plan" gpurun_out/r04aa_bench_plan_$i.err | tail -3
done
