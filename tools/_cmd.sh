set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_resize.py tests/test_gpu_jpeg.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
timeout -k 10 200 python -u bench.py --config stage --steps 10 --no-cpu-baseline > gpurun_out/r02u_bench_stage.json
timeout -k 10 300 python -u bench.py --config jpeg --steps 10 --no-cpu-baseline > gpurun_out/jpeg_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stage -- python3 -u bench.py --config stage --steps 5 --no-cpu-baseline > /dev/null
find gpurun_out/prof_stage -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/stage_kernel_stats.csv
