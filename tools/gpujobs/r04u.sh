set -o pipefail
cd $GRAFT_REPO_ROOT
WICCA_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/v_ck32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 120 --timeout-method thread -k "golden or corpus or variants or damage or corrupt" > gpurun_out/r04u_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04u_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 8 16 32 8 16 32; do
  if [ $v = 8 ]; then L=$GRAFT_REPO_ROOT/wicca_amd/libwicca_hip.so; else L=$GRAFT_REPO_ROOT/tools/bin/v_ck$v.so; fi
  rm -rf gpurun_out/prof_r04u_ck$v
  WICCA_HIP_LIB=$L bash tools/profile_bench.sh r04u_ck$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "cks=$v $(grep 'sync_kernel\|write_kernel' gpurun_out/prof_r04u_ck$v/kstats.txt | awk '{printf "%s/%s | ", $1, $2}')"
done
