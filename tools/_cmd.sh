set -e
timeout -k 10 300 python -u bench.py > gpurun_out/r02u_bench_default.json 2> gpurun_out/r02u_bench_default.err
cat gpurun_out/r02u_bench_default.json
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash tools/profile_gpu.sh r02u
cat gpurun_out/prof_r02u/summary.json
