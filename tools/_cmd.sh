set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
tail -1 gpurun_out/gpu_suite.log
timeout -k 10 300 python -u bench.py --config multi --depths 2,3,4,5,6 --steps 10 --no-cpu-baseline > gpurun_out/bench_multi26.json
timeout -k 10 300 python -u bench.py --config multi --depths 1,2,3,4,5,6 --steps 10 --no-cpu-baseline > gpurun_out/bench_multi16.json
for f in multi26 multi16; do python3 -c "import json,sys; j=json.load(open('gpurun_out/bench_$f.json')); print('$f', j['ms_per_step'], j['roofline']['achieved'], j['roofline']['frac'])"; done
