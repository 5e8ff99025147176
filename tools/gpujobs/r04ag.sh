set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 4096 5120 6144 4096 5120 6144; do
  rm -rf gpurun_out/prof_r04ag_s$b
  WICCA_JPEG_SUB_BITS=$b bash tools/profile_bench.sh r04ag_s$b --config jpeg --steps 4 --warmup 1 > /dev/null || exit 1
  echo "sub_bits=$b $(python3 tools/gpujobs/huff_sum.py gpurun_out/prof_r04ag_s$b/kstats.txt) $(grep -o '"value": [0-9.]*' gpurun_out/prof_r04ag_s$b/bench.log | head -1)"
done
