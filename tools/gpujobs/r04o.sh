set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_jpeg_idct.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04o_tests.log
[ $rc -eq 0 ] || exit $rc
for v in pd1 pd4; do
  if [ $v = pd1 ]; then L=$GRAFT_REPO_ROOT/tools/bin/v_pd1.so; else L=$GRAFT_REPO_ROOT/wicca_amd/libwicca_hip.so; fi
  WICCA_HIP_LIB=$L bash tools/profile_bench.sh r04o_$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "$v $(grep 'write_kernel\|sync_kernel' gpurun_out/prof_r04o_$v/kstats.txt | awk '{printf "%s/%s/%s | ", $1, $2, $3}')"
  WICCA_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config jpeg --steps 6 --warmup 2 > gpurun_out/r04o_bench_$v.json 2> /dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04o_bench_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['unit'], d['ms_per_step'])"
done
