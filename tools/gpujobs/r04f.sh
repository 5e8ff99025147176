set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/diag/jpeg_damage_diag.py > gpurun_out/r04f_damage.txt 2>&1; cat gpurun_out/r04f_damage.txt
C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
bash tools/pmc_bench.sh r04f_plan_wait "$C" --config plan --steps 1 --warmup 0 --plan-no-loop --no-verify || exit 1
grep -A9 "plan_rows\|haar_multi_rag" gpurun_out/pmc_r04f_plan_wait/summary.txt
bash tools/pmc_bench.sh r04f_jpeg_wait "$C" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
grep -A9 "stage_rows\|luma_color" gpurun_out/pmc_r04f_jpeg_wait/summary.txt
timeout -k 10 240 tools/bin/hbm_probe c > gpurun_out/r04f_hbm_probe.txt 2>&1; head -14 gpurun_out/r04f_hbm_probe.txt
