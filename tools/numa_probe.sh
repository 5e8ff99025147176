set -e
mkdir -p gpurun_out
{ rocm-smi --showtoponuma 2>&1 | grep -i numa || true; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done; which taskset numactl || true; } > gpurun_out/r06w_numa.txt 2>&1
NODE=$(rocm-smi --showtoponuma 2>/dev/null | grep -i "numa node" | head -1 | sed 's/.*: *//' | tr -dc '0-9')
CPUS=$(cat /sys/devices/system/node/node${NODE:-0}/cpulist)
echo "gpu node $NODE cpus $CPUS" >> gpurun_out/r06w_numa.txt
timeout -k 10 300 taskset -c "$CPUS" python -u tools/plan_variance_probe.py 5 12 > gpurun_out/r06w_plan_variance_bound.txt 2>&1
timeout -k 10 300 python -u tools/plan_variance_probe.py 5 12 > gpurun_out/r06w_plan_variance_free.txt 2>&1
