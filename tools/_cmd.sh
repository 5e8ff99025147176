set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
timeout -k 10 300 python -u bench.py --config jpeg --steps 10 --no-cpu-baseline > gpurun_out/jpeg_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jpeg -- python3 -u bench.py --config jpeg --steps 5 --no-cpu-baseline > gpurun_out/jpeg_prof.json
find gpurun_out/prof_jpeg -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/jpeg_kernel_stats.csv
find gpurun_out/prof_jpeg -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/jpeg_kernel_trace.csv
