# Timing-only: the write pass without its block stores (wrong coefficients),
# to see how much of it the stores' share of the load counter costs.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in full nostore full nostore; do
  rm -rf gpurun_out/prof_r04ak_$v
  if [ $v = full ]; then unset WICCA_HIP_LIB; else export WICCA_HIP_LIB=$GRAFT_REPO_ROOT/tools/bin/libwicca_nostore.so; fi
  bash tools/profile_bench.sh r04ak_$v --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "$v $(python3 tools/gpujobs/huff_sum.py gpurun_out/prof_r04ak_$v/kstats.txt)"
done
