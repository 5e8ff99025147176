set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -q -x --timeout 120 --timeout-method thread -k "stage or fused" > gpurun_out/r04l_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r04l_tests.log
[ $rc -eq 0 ] || exit $rc
WICCA_STAGE_PARTS=0 bash tools/profile_bench.sh r04l_whole --config jpeg --steps 4 --warmup 1 > /dev/null || exit 1
bash tools/profile_bench.sh r04l_parts --config jpeg --steps 4 --warmup 1 > /dev/null || exit 1
for v in whole parts; do echo "$v $(grep 'stage_rows\|luma_color' gpurun_out/prof_r04l_$v/kstats.txt | awk '{printf "%s %s %s | ", $3, $4, $NF}')"; tail -1 gpurun_out/prof_r04l_$v/bench.log | cut -c1-300; done
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
bash tools/pmc_bench.sh r04l_parts_sq "$C" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
grep -A9 "stage_rows" gpurun_out/pmc_r04l_parts_sq/summary.txt
bash tools/pmc_bench.sh r04l_parts_fetch "FETCH_SIZE" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
bash tools/pmc_bench.sh r04l_parts_write "WRITE_SIZE" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
grep -A2 "stage_rows" gpurun_out/pmc_r04l_parts_fetch/summary.txt gpurun_out/pmc_r04l_parts_write/summary.txt
