#!/bin/bash
# What the GPU box offers the CPU baseline: CPU model, affinity, cgroup CPU quota, OMP setting.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
{
  echo "model: $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2-)"
  echo "nproc: $(nproc)"
  python3 -c "import os; print('affinity:', len(os.sched_getaffinity(0)), 'cpu_count:', os.cpu_count())"
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo none)"
  echo "cpuset.cpus.effective: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || echo none)"
  echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset} MAX_JOBS=${MAX_JOBS:-unset}"
  grep -E 'MemTotal' /proc/meminfo
} > gpurun_out/box_probe.txt 2>&1
cat gpurun_out/box_probe.txt
