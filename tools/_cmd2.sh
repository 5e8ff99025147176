set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
WICCA_JPEG_TIMING=1 timeout -k 10 300 python -u bench.py --config jpeg --steps 10 --no-cpu-baseline > gpurun_out/jpeg_bench.json 2> gpurun_out/jpeg_bench.err
tail -1 gpurun_out/jpeg_bench.err
