#!/bin/bash
# Round 6: host placement probe for the producer's encode (NUMA nodes, cgroup quota), then the
# encode under no pinning, and pinned to 16 CPUs of each NUMA node. Outputs gpurun_out/r06k/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06k
mkdir -p $O
{ lscpu | grep -E "Model name|Socket|NUMA|Thread|Core"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; } > $O/topology.txt 2>&1
timeout -k 10 120 python -u tools/numa_probe.py > $O/enc_free.log 2>&1 || exit $?
for node in $(lscpu | awk -F: '/NUMA node[0-9]+ CPU/ {print $1}' | grep -o '[0-9]\+' | head -4); do
  cl=$(lscpu | awk -F: "/NUMA node$node CPU/ {print \$2}" | tr -d ' ' | cut -d, -f1)
  lo=${cl%-*}
  timeout -k 10 120 taskset -c $lo-$((lo + 15)) python -u tools/numa_probe.py > $O/enc_node$node.log 2>&1 || exit $?
done
cat $O/enc_*.log
echo all ok
