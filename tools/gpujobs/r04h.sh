set -o pipefail
cd $GRAFT_REPO_ROOT
WICCA_JPEG_TIMING=1 timeout -k 10 120 python -u tools/diag/jpeg_corrupt_diag.py > gpurun_out/r04h_corrupt.txt 2>&1; rc0=$?; grep -v "parse+destuff" gpurun_out/r04h_corrupt.txt | tail -20
[ $rc0 -eq 0 ] || exit $rc0
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -q --timeout 120 --timeout-method thread -rs > gpurun_out/r04h_tests.log 2>&1; rc=$?; tail -8 gpurun_out/r04h_tests.log
[ $rc -le 1 ] || exit $rc
bash tools/profile_bench.sh r04h_jpeg --config jpeg --steps 5 --warmup 2 || exit 1
grep -B2 -A12 "total_ms" gpurun_out/prof_r04h_jpeg/kstats.txt | head -16
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"
bash tools/pmc_bench.sh r04h_luma "$C" --config jpeg --steps 2 --warmup 1 --no-verify || exit 1
grep -A7 "luma_color\|jpeg_idct" gpurun_out/pmc_r04h_luma/summary.txt
exit $rc
