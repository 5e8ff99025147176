set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
tail -1 gpurun_out/gpu_suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()"
