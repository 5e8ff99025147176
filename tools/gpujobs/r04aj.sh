# End-of-round-4 run (after the interleaved stream layout): the whole GPU
# suite, smoke, the default bench and the JPEG / plan legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=r04aj
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -rs > gpurun_out/${T}_gputest_full.txt 2>&1; rc=$?; tail -3 gpurun_out/${T}_gputest_full.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1; rc=$?; tail -1 gpurun_out/${T}_smoke.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err; rc=$?; grep -o '"value": [0-9.]*\|"frac": [0-9.]*' gpurun_out/${T}_bench_default.json | head -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config jpeg > gpurun_out/${T}_bench_jpeg.json 2> gpurun_out/${T}_bench_jpeg.err || exit 1
grep -o '"value": [0-9.]*' gpurun_out/${T}_bench_jpeg.json | head -1
timeout -k 10 600 python -u bench.py --config plan > gpurun_out/${T}_bench_plan.json 2> gpurun_out/${T}_bench_plan.err || exit 1
grep -o '"value": [0-9.]*' gpurun_out/${T}_bench_plan.json | head -1
echo done
