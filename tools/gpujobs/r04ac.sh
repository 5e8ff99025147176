set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_jpeg_idct.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04ac_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04ac_tests.log
[ $rc -eq 0 ] || exit $rc
WICCA_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libwicca_r4c8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 180 --timeout-method thread -k "golden or corpus or damage or corrupt or trunc or restart" > gpurun_out/r04ac_tests_c8.log 2>&1; rc=$?; tail -1 gpurun_out/r04ac_tests_c8.log
[ $rc -eq 0 ] || exit $rc
for v in new old c8 new old c8; do
  rm -rf gpurun_out/prof_r04ac_$v
  if [ $v = new ]; then unset WICCA_HIP_LIB; else export WICCA_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libwicca_r4$v.so; fi
  bash tools/profile_bench.sh r04ac_$v --config jpeg --steps 4 --warmup 1 > /dev/null || exit 1
  echo "$v $(python3 tools/gpujobs/huff_sum.py gpurun_out/prof_r04ac_$v/kstats.txt) $(grep -o '"value": [0-9.]*' gpurun_out/prof_r04ac_$v/bench.log | head -1)"
done
unset WICCA_HIP_LIB
bash tools/pmc_bench.sh r04ac_fetch "FETCH_SIZE" --config jpeg --steps 1 --warmup 0 --no-verify > /dev/null || exit 1
grep -A1 "sync_kernel<1\|write_kernel" gpurun_out/pmc_r04ac_fetch/summary.txt
