# SQ wait ratios of the JPEG kernels after the interleaved stream layout.
set -o pipefail
cd $GRAFT_REPO_ROOT
C="SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT"
bash tools/pmc_bench.sh r04am_jpeg_sq "$C" --config jpeg --steps 1 --warmup 0 --no-verify > /dev/null || exit 1
echo done
