set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_nest -- python3 -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/bench_nested.json
python3 -c "import json; j=json.load(open('gpurun_out/bench_nested.json')); print(j['roofline']['pmc_source'], j['roofline']['traffic'])"
