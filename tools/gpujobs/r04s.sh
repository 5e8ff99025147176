set -o pipefail
cd $GRAFT_REPO_ROOT
WICCA_JPEG_TIMING=1 timeout -k 10 400 python -u bench.py --config plan --steps 3 --warmup 1 --plan-no-loop > gpurun_out/r04s_plan.json 2> gpurun_out/r04s_plan.err; rc=$?
grep "wicca plan\|device decode" gpurun_out/r04s_plan.err | tail -6; tail -c 600 gpurun_out/r04s_plan.json
exit $rc
