set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 2048 3072 4096 6144 2048 4096; do
  rm -rf gpurun_out/prof_r04x_s$b
  WICCA_JPEG_SUB_BITS=$b bash tools/profile_bench.sh r04x_s$b --config jpeg --steps 4 --warmup 1 > /dev/null || exit 1
  echo "sub_bits=$b $(python3 tools/gpujobs/huff_sum.py gpurun_out/prof_r04x_s$b/kstats.txt) $(grep -o '"value": [0-9.]*' gpurun_out/prof_r04x_s$b/bench.log | head -1)"
done
