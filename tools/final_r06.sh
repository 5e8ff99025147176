#!/bin/bash
# Round-6 final evidence on the GPU box: full GPU suite, smoke, headline / JPEG / plan benches, JPEG kernel trace.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06g_gputest_full.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06g_smoke.txt 2>&1
timeout -k 10 240 python -u bench.py > gpurun_out/r06g_bench_headline.json 2> gpurun_out/r06g_bench_headline.err
timeout -k 10 240 python -u bench.py --config jpeg > gpurun_out/r06g_bench_jpeg.json 2> gpurun_out/r06g_bench_jpeg.err
timeout -k 10 300 python -u bench.py --config plan > gpurun_out/r06g_bench_plan.json 2> gpurun_out/r06g_bench_plan.err
bash tools/profile_jpeg.sh r06g_jpeg > /dev/null 2>&1
echo "final done"
