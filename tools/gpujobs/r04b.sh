set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py -k "gif" tests/test_gpu_jpeg.py::test_async_decode_matches_libjpeg tests/test_gpu_jpeg.py::test_file_stage_pipelined_matches_synchronous -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 || { tail -30 gpurun_out/r04b_tests.log; exit 1; }
tail -3 gpurun_out/r04b_tests.log
bash tools/profile_bench.sh r04b_plan --config plan --steps 3 --warmup 1 --plan-no-loop || exit 1
cat gpurun_out/prof_r04b_plan/kstats.txt | head -30
bash tools/pmc_bench.sh r04b_plan_sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" --config plan --steps 1 --warmup 0 --plan-no-loop --no-verify || exit 1
bash tools/pmc_bench.sh r04b_plan_hbm "FETCH_SIZE" --config plan --steps 1 --warmup 0 --plan-no-loop --no-verify || exit 1
bash tools/pmc_bench.sh r04b_plan_wr "WRITE_SIZE" --config plan --steps 1 --warmup 0 --plan-no-loop --no-verify || exit 1
bash tools/pmc_bench.sh r04b_jpeg_sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
head -80 gpurun_out/pmc_r04b_plan_sq/summary.txt
