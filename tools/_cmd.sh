set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
tail -1 gpurun_out/gpu_suite.log
R3="--config ragged --depth 3 --images 256 --height 2160 --width 3840 --ragged-align 128 --steps 30 --no-cpu-baseline"
R5="--config ragged --depth 5 --images 128 --ragged-align 128 --steps 20 --no-cpu-baseline"
timeout -k 10 120 python -u bench.py $R3 > gpurun_out/r02_bench_ragged_d3.json
timeout -k 10 120 python -u bench.py $R5 > gpurun_out/r02_bench_ragged_d5.json
timeout -k 10 120 python -u bench.py --config ragged --depth 1 --images 256 --height 2160 --width 3840 --ragged-align 128 --steps 30 --no-cpu-baseline > gpurun_out/r02_bench_ragged_d1.json
timeout -k 10 120 python -u bench.py --config ragged --depth 2 --images 256 --height 2160 --width 3840 --ragged-align 128 --steps 30 --no-cpu-baseline > gpurun_out/r02_bench_ragged_d2.json
cat gpurun_out/r02_bench_ragged_d*.json
