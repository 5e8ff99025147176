set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "multi" 2>&1 | tail -1
timeout -k 10 100 python -u bench.py --config multi --depths 1,2,3,4,5,6 --steps 10 --no-cpu-baseline > gpurun_out/r02u_bench_multi16.json
timeout -k 10 100 python -u bench.py --config multi --depths 2,3,4,5,6 --steps 10 --no-cpu-baseline > gpurun_out/r02u_bench_multi26.json
python3 -c "import json; [print(f, json.load(open('gpurun_out/'+f))['ms_per_step']) for f in ('r02u_bench_multi16.json','r02u_bench_multi26.json')]"
