set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
tail -1 gpurun_out/gpu_suite.log
for d in 1 4; do
timeout -k 10 300 python -u bench.py --config ragged --depth $d --images 256 --height 2160 --width 3840 --ragged-align 128 --steps 30 --no-cpu-baseline > gpurun_out/bench_ragged_d$d.json
cat gpurun_out/bench_ragged_d$d.json | python3 -c "import json,sys; j=json.load(sys.stdin); print($d, j['ms_per_step'], j['roofline']['achieved'], j['roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --depth 1 --no-cpu-baseline > gpurun_out/bench_u_d1.json
cat gpurun_out/bench_u_d1.json | python3 -c "import json,sys; j=json.load(sys.stdin); print('u1', j['ms_per_step'], j['roofline']['achieved'], j['roofline']['frac'])"
