#!/bin/bash
# Host facts of the GPU box that the CPU baseline depends on.
python -c "import os; print('os.cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"
echo "nproc $(nproc)"; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
grep -m1 "model name" /proc/cpuinfo || true
free -g | head -2
