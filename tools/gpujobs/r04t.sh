set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_jpeg_idct.py tests/test_gpu_plan.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04t_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 2 1 2; do
  WICCA_JPEG_SYNC_CK=$v bash tools/profile_bench.sh r04t_ck$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "ck=$v $(grep 'sync_kernel\|write_kernel' gpurun_out/prof_r04t_ck$v/kstats.txt | awk '{printf "%s/%s | ", $1, $2}')"
done
WICCA_JPEG_TIMING=1 timeout -k 10 300 python -u bench.py --config jpeg --steps 3 --warmup 1 > gpurun_out/r04t_bench.json 2> gpurun_out/r04t_bench.err || exit 1
grep "checkpoint hits" gpurun_out/r04t_bench.err | tail -2; python3 -c "import json;d=json.loads(open('gpurun_out/r04t_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['unit'],d['ms_per_step'])"
