#!/bin/bash
# Diagnostics: the box's NUMA layout, the CPUs this process may use and the GPU's node.
echo "allowed: $(python3 -c 'import os; s=sorted(os.sched_getaffinity(0)); print(len(s), s[:8], s[-8:])')"
ls /sys/devices/system/node/ | grep node
for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done
for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d numa=$(cat $d/numa_node) vendor=$(cat $d/vendor 2>/dev/null)"; done
python3 - <<'PY'
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
buf = ctypes.create_string_buffer(64)
n = ctypes.c_int()
hip.hipGetDeviceCount(ctypes.byref(n)); print("devices", n.value)
hip.hipDeviceGetPCIBusId(buf, 64, 0); print("pci", buf.value)
PY
which numactl || true
python3 - <<'PY'
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
buf = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(buf, 64, 0)
bus = buf.value.decode().lower()
print("gpu", bus, "numa_node", open("/sys/bus/pci/devices/%s/numa_node" % bus).read().strip())
PY
