#!/bin/bash
# Round-4 session V: the slow trace_rays_batch mode -- the probe pinned (taskset, before any GPU
# use) to each NUMA node's CPUs, after a host-frame leg, several processes each.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for f in /sys/class/drm/renderD*/device/numa_node; do echo "$f $(cat $f)"; done | head -12
ls /sys/devices/system/node/ | grep node
for node in 0 1; do
  cpus=$(cat /sys/devices/system/node/node$node/cpulist 2>/dev/null) || continue
  [ -n "$cpus" ] || continue
  for r in 1 2 3; do
    WHERE=1 PRE_FRAMES=1 CHUNKS=x timeout -k 10 200 taskset -c "$cpus" python3 tools/batch_probe.py > $OUT/bp.txt 2> /dev/null || { echo "probe failed"; exit 1; }
    echo "node $node: $(grep -v 'num_threads 8' $OUT/bp.txt | tr '\n' ' ')"
  done
done
for r in 1 2 3; do
  WHERE=1 PRE_FRAMES=1 CHUNKS=x timeout -k 10 200 python3 tools/batch_probe.py > $OUT/bp.txt 2> /dev/null || { echo "probe failed"; exit 1; }
  echo "free: $(grep -v 'num_threads 8' $OUT/bp.txt | tr '\n' ' ')"
done
echo all-done
