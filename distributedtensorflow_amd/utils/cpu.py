"""CPUs this process may actually use.

``os.cpu_count()`` reports every CPU of the machine.  On a shared GPU host (one container slice of
a many-core node) a process that sizes its thread pools by it -- as the reference does with
``intra_op_parallelism_threads=os.cpu_count()`` (``run_mnist_distributed.py:122-124``) --
oversubscribes its CPU quota many times over.  :func:`usable_cpus` is the tightest of: the
scheduler affinity mask, the cgroup CPU quota (v2 ``cpu.max`` / v1 ``cfs_quota_us``) and an
explicit ``OMP_NUM_THREADS``.
"""
from __future__ import annotations

import math
import os


def _cgroup_quota():
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
            if quota != "max":
                return max(1, math.ceil(int(quota) / int(period)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            quota = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = int(f.read())
        if quota > 0 and period > 0:
            return max(1, math.ceil(quota / period))
    except (OSError, ValueError):
        pass
    return None


def usable_cpus() -> int:
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    q = _cgroup_quota()
    if q:
        n = min(n, q)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)
