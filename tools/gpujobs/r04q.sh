set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 1 2 4 8 3 15; do
  WICCA_JPEG_ABL=$a bash tools/profile_bench.sh r04q_abl$a --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "abl=$a $(grep luma_color gpurun_out/prof_r04q_abl$a/kstats.txt | awk '{print $3, $4}')"
done
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
bash tools/pmc_bench.sh r04q_luma "$C" --config jpeg --steps 1 --warmup 0 --no-verify || exit 1
grep -A9 "luma_color" gpurun_out/pmc_r04q_luma/summary.txt
