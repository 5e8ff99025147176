set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 2 4; do
WICCA_JPEG_LUMA_ROWS=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 120 --timeout-method thread -k "golden or corpus or fused or orient or extreme or stage" > gpurun_out/r04w_tests_$r.log 2>&1; rc=$?; tail -1 gpurun_out/r04w_tests_$r.log
[ $rc -eq 0 ] || exit $rc
done
for v in 1 2 4 1 2 4; do
  rm -rf gpurun_out/prof_r04w_r$v
  WICCA_JPEG_LUMA_ROWS=$v bash tools/profile_bench.sh r04w_r$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "rows=$v $(grep 'luma_color' gpurun_out/prof_r04w_r$v/kstats.txt | awk '{print $3, $4}')"
done
