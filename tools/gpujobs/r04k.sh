set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # tag lib env...
  t=$1; L=$2; shift 2
  env "$@" WICCA_HIP_LIB=$L bash tools/profile_bench.sh r04k_$t --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "$t $(grep 'luma_color\|jpeg_idct' gpurun_out/prof_r04k_$t/kstats.txt | awk '{print $3, $4}' | tr '\n' ' ')"
}
B=$GRAFT_REPO_ROOT/wicca_amd/libwicca_hip.so
run base $B X=1
run nt $GRAFT_REPO_ROOT/tools/bin/v_nt.so X=1
run w8 $GRAFT_REPO_ROOT/tools/bin/v_w8.so X=1
run xt2 $B WICCA_JPEG_XT=2
run xt4 $B WICCA_JPEG_XT=4
run xt8 $B WICCA_JPEG_XT=8
run base2 $B X=1
for a in 1 2 4 7; do
  WICCA_STAGE_ABL=$a bash tools/profile_bench.sh r04k_sabl$a --config jpeg --steps 4 --warmup 1 --no-verify > /dev/null || exit 1
  echo "stage_abl=$a $(grep 'stage_rows' gpurun_out/prof_r04k_sabl$a/kstats.txt | awk '{print $3, $4}' | tr '\n' ' ')"
done
echo "base stage $(grep 'stage_rows' gpurun_out/prof_r04k_base/kstats.txt | awk '{print $3, $4}')"
timeout -k 10 240 tools/bin/hbm_probe c > gpurun_out/r04k_hbm_probe.txt 2>&1; grep "flat" gpurun_out/r04k_hbm_probe.txt
