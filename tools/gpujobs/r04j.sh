set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 1 2 4 8 3 15; do
  WICCA_JPEG_ABL=$a bash tools/profile_bench.sh r04j_abl$a --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "abl=$a $(grep luma_color gpurun_out/prof_r04j_abl$a/kstats.txt | awk '{print $3, $4}')"
done
