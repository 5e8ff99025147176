set -e
start=$(date +%s)
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.json
echo "bench wall $(( $(date +%s) - start )) s"
cat gpurun_out/bench_default.json
