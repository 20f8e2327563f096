#!/bin/bash
# Does the host's NUMA placement matter for the host-side paths?  The box has 2 NUMA nodes
# (lscpu: node0 = CPUs 0-63,128-191, node1 = 64-127,192-255) and the container may run on any
# of its 256 CPUs (16 CPUs of quota).  scripts/ck_host_cost (quick: CPU path, GPU route, the
# split) runs unpinned, on the GPU's node and on the other node -- each run writes its files
# from its own threads, so the page cache lands on the node it runs on.
set -u
mkdir -p gpurun_out
dev=$(python3 - <<'PY'
import ctypes
buf = ctypes.create_string_buffer(64)
ctypes.CDLL("libamdhip64.so").hipDeviceGetPCIBusId(buf, 64, 0)
print(buf.value.decode().lower())
PY
)
node=$(cat /sys/bus/pci/devices/$dev/numa_node 2>/dev/null || echo -1)
echo "gpu $dev numa_node $node" | tee gpurun_out/numa.txt
cat /sys/devices/system/node/node0/cpulist /sys/devices/system/node/node1/cpulist >> gpurun_out/numa.txt
local_cpus=$(cat /sys/devices/system/node/node$([ "$node" = 1 ] && echo 1 || echo 0)/cpulist)
remote_cpus=$(cat /sys/devices/system/node/node$([ "$node" = 1 ] && echo 0 || echo 1)/cpulist)
for where in unpinned local remote; do
  case $where in
    unpinned) pre="";;
    local) pre="taskset -c $local_cpus";;
    remote) pre="taskset -c $remote_cpus";;
  esac
  echo "== $where" >> gpurun_out/numa.txt
  timeout -k 10 200 $pre ./scripts/ck_host_cost 32 256 2.4 quick >> gpurun_out/numa.txt 2>&1
  rc=$?; echo "$where rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/numa.txt
