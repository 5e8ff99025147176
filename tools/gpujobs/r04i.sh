set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_jpeg_idct.py -q --timeout 120 --timeout-method thread -rs > gpurun_out/r04i_tests.log 2>&1; rc=$?; tail -6 gpurun_out/r04i_tests.log
[ $rc -le 1 ] || exit $rc
WICCA_JPEG_TIMING=1 timeout -k 10 120 python -u tools/diag/jpeg_corrupt_diag.py 3 4 2>&1 | grep -v "parse+destuff\|subsequences" 
WICCA_JPEG_XCD=0 bash tools/profile_bench.sh r04i_jpeg_noxcd --config jpeg --steps 5 --warmup 2 || exit 1
bash tools/profile_bench.sh r04i_jpeg_xcd --config jpeg --steps 5 --warmup 2 || exit 1
for v in noxcd xcd; do echo "== $v"; grep "luma_color\|jpeg_idct" gpurun_out/prof_r04i_jpeg_$v/kstats.txt; done
C="FETCH_SIZE TCC_HIT_sum"
WICCA_JPEG_XCD=0 bash tools/pmc_bench.sh r04i_fetch_noxcd "$C" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
bash tools/pmc_bench.sh r04i_fetch_xcd "$C" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
for v in noxcd xcd; do echo "== $v"; grep -A3 "luma_color" gpurun_out/pmc_r04i_fetch_$v/summary.txt; done
exit $rc
