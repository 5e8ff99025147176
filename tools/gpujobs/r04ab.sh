# End-of-round PMC of the JPEG and plan kernels (one SQ pass each, then a
# FETCH/WRITE pass): the wait ratios and instruction counts of the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
C="SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT"
bash tools/pmc_bench.sh r04ab_jpeg_sq "$C" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
bash tools/pmc_bench.sh r04ab_plan_sq "$C" --config plan --steps 1 --warmup 0 --plan-no-loop --no-verify || exit 1
bash tools/pmc_bench.sh r04ab_jpeg_fetch "FETCH_SIZE" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
bash tools/pmc_bench.sh r04ab_jpeg_write "WRITE_SIZE" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
grep -c . gpurun_out/pmc_r04ab_jpeg_sq/summary.txt
