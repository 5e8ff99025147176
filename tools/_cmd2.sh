set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
tail -1 gpurun_out/gpu_suite.log
WICCA_JPEG_TIMING=1 timeout -k 10 300 python -u bench.py --config jpeg --steps 10 --no-cpu-baseline > gpurun_out/jpeg_bench.json 2> gpurun_out/jpeg_bench.err
tail -1 gpurun_out/jpeg_bench.err
