# End-of-round-4 run: the whole GPU suite, smoke, the default bench (live PMC),
# a rocprofv3 kernel summary of the default bench, and the JPEG / plan legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=r04z
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -rs > gpurun_out/${T}_gputest_full.txt 2>&1; rc=$?; tail -4 gpurun_out/${T}_gputest_full.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1; rc=$?; tail -1 gpurun_out/${T}_smoke.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err; rc=$?; tail -c 600 gpurun_out/${T}_bench_default.json
[ $rc -eq 0 ] || exit $rc
bash tools/profile_bench.sh ${T}_default --steps 20 --warmup 3 --no-live-pmc > /dev/null || exit 1
head -4 gpurun_out/prof_${T}_default/kstats.txt
timeout -k 10 600 python -u bench.py --config jpeg > gpurun_out/${T}_bench_jpeg.json 2> gpurun_out/${T}_bench_jpeg.err || exit 1
timeout -k 10 600 python -u bench.py --config plan > gpurun_out/${T}_bench_plan.json 2> gpurun_out/${T}_bench_plan.err || exit 1
echo done
