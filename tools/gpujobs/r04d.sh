set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_jpeg.py -k "plan or stage" -x -q --timeout 180 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1 || { tail -30 gpurun_out/r04d_tests.log; exit 1; }
tail -3 gpurun_out/r04d_tests.log
bash tools/profile_bench.sh r04d_plan --config plan --steps 3 --warmup 1 --plan-no-loop || exit 1
head -20 gpurun_out/prof_r04d_plan/kstats.txt
bash tools/profile_bench.sh r04d_jpeg --config jpeg --steps 3 --warmup 1 || exit 1
head -14 gpurun_out/prof_r04d_jpeg/kstats.txt
bash tools/pmc_bench.sh r04d_plan_sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" --config plan --steps 1 --warmup 0 --plan-no-loop --no-verify || exit 1
grep -A7 "plan_rows" gpurun_out/pmc_r04d_plan_sq/summary.txt
bash tools/pmc_bench.sh r04d_jpeg_sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
grep -A7 "stage_rows" gpurun_out/pmc_r04d_jpeg_sq/summary.txt
timeout -k 10 300 python -u bench.py --config plan --steps 3 --warmup 1 > gpurun_out/r04d_plan.json 2> gpurun_out/r04d_plan.err || exit 1
cat gpurun_out/r04d_plan.json
