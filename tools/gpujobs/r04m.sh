set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 120 --timeout-method thread -k "stage or fused" > gpurun_out/r04m_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04m_tests.log
[ $rc -eq 0 ] || exit $rc
for a in 0 8; do
  WICCA_STAGE_PARTS=0 WICCA_STAGE_ABL=$a bash tools/profile_bench.sh r04m_w$a --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  WICCA_STAGE_ABL=$a bash tools/profile_bench.sh r04m_p$a --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "abl=$a whole $(grep 'stage_rows' gpurun_out/prof_r04m_w$a/kstats.txt | awk '{print $3}')  parts $(grep 'stage_rows' gpurun_out/prof_r04m_p$a/kstats.txt | awk '{print $3}')"
done
