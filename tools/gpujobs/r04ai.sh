set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_jpeg_idct.py tests/test_gpu_plan.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04ai_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04ai_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  rm -rf gpurun_out/prof_r04ai_i$v
  WICCA_JPEG_ILV=$v bash tools/profile_bench.sh r04ai_i$v --config jpeg --steps 4 --warmup 1 > /dev/null || exit 1
  echo "ilv=$v $(python3 tools/gpujobs/huff_sum.py gpurun_out/prof_r04ai_i$v/kstats.txt) $(grep 'interleave' gpurun_out/prof_r04ai_i$v/kstats.txt | awk '{print "ilv_us", $3}') $(grep -o '"value": [0-9.]*' gpurun_out/prof_r04ai_i$v/bench.log | head -1)"
done
bash tools/pmc_bench.sh r04ai_fetch "FETCH_SIZE" --config jpeg --steps 1 --warmup 0 --no-verify > /dev/null || exit 1
grep -A1 "sync_kernel<1\|write_kernel\|sync_kernel<3" gpurun_out/pmc_r04ai_fetch/summary.txt
