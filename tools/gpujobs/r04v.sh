set -o pipefail
cd $GRAFT_REPO_ROOT
WICCA_JPEG_DIRECT_RGB=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_jpeg_idct.py -q -x --timeout 120 --timeout-method thread -k "golden or corpus or fused or orient or extreme or stage" > gpurun_out/r04v_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04v_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 2 1 2; do
  rm -rf gpurun_out/prof_r04v_d$v
  WICCA_JPEG_DIRECT_RGB=$v bash tools/profile_bench.sh r04v_d$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "direct=$v $(grep 'luma_color' gpurun_out/prof_r04v_d$v/kstats.txt | awk '{print $3, $4}')"
done
