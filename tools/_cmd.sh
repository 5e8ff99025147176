set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in r1 r2 r4; do
WICCA_HIP_LIB=tools/variants/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c_$v -- python3 -u bench.py --config jpeg --steps 5 --no-cpu-baseline > gpurun_out/jpeg_c_$v.json
f=$(find gpurun_out/prof_c_$v -name "*kernel_stats.csv" | head -1); grep color $f | cut -d, -f1-5 | sed "s/^/$v /"
done
