set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plan.py -x -q --timeout 120 --timeout-method thread -rs > gpurun_out/r04g_tests.log 2>&1; rc=$?; tail -25 gpurun_out/r04g_tests.log
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"
bash tools/pmc_bench.sh r04g_full "$C" --config jpeg --steps 2 --warmup 1 --no-verify || exit 1
WICCA_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/abl_noidct.so bash tools/pmc_bench.sh r04g_noidct "$C" --config jpeg --steps 2 --warmup 1 --no-verify || exit 1
WICCA_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/abl_nocolor.so bash tools/pmc_bench.sh r04g_nocolor "$C" --config jpeg --steps 2 --warmup 1 --no-verify || exit 1
for v in full noidct nocolor; do echo "== $v"; grep -A7 "luma_color" gpurun_out/pmc_r04g_$v/summary.txt; done
exit $rc
