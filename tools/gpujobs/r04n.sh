set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -rs > gpurun_out/r04n_gputest_full.txt 2>&1; rc=$?; tail -8 gpurun_out/r04n_gputest_full.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04n_smoke.txt 2>&1; rc=$?; tail -3 gpurun_out/r04n_smoke.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04n_bench_default.json 2> gpurun_out/r04n_bench_default.err; rc=$?; tail -c 1500 gpurun_out/r04n_bench_default.json
exit $rc
