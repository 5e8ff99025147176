set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0 1; do
  WICCA_JPEG_DIRECT_RGB=$v bash tools/profile_bench.sh r04r_d$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "direct=$v $(grep 'luma_color' gpurun_out/prof_r04r_d$v/kstats.txt | awk '{print $3, $4}')"
done
