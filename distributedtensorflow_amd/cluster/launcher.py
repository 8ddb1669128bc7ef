"""Local cluster launcher: start every task of a PS/worker cluster as its own process.

The reference starts each task by hand (``python run_mnist_distributed.py --job_name=ps
--task_index=0`` on every host; README).  ``launch_local`` does the same on one host: it writes a
``config.json`` (127.0.0.1, free ports), spawns ``num_ps`` PS and ``num_workers`` worker
processes of ``script``, streams their logs to files, waits for the workers, and makes sure the
PS processes exit (they return from ``join()`` when all workers stopped; anything still alive
after ``grace_s`` is terminated by PID — never by pattern).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def write_config(path, num_ps, num_workers):
    ports = free_ports(num_ps + num_workers)
    cfg = {"ps": {f"ps:{i}": f"127.0.0.1:{ports[i]}" for i in range(num_ps)},
           "workers": {f"worker:{i}": f"127.0.0.1:{ports[num_ps + i]}"
                       for i in range(num_workers)}}
    with open(path, "w") as f:
        json.dump(cfg, f, indent=2)
    return cfg


def _cleanup_shm(pid):
    """/dev/shm segments a killed PS task left behind (names carry the owner's pid)."""
    import glob
    for f in glob.glob(f"/dev/shm/dtf_*_{pid}_*"):
        try:
            os.unlink(f)
        except OSError:
            pass


def launch_local(script, num_ps=1, num_workers=2, workdir=None, extra_args=(), env=None,
                 timeout_s=600, grace_s=30, gpus_per_host=None, max_ps_restarts=0):
    """``max_ps_restarts``: a PS task that dies (non-zero exit, e.g. killed) while workers are
    still running is restarted as a FRESH process (same flags, ``DTF_RESTART_COUNT`` set) up
    to this many times; it rejoins the next process-group generation and the workers recover
    from the latest checkpoint (MonitoredTrainingSession)."""
    workdir = os.path.abspath(workdir or os.getcwd())
    script = os.path.abspath(script)          # tasks run with cwd=workdir
    os.makedirs(workdir, exist_ok=True)
    cfg_path = os.path.join(workdir, "config.json")
    write_config(cfg_path, num_ps, num_workers)
    base_env = dict(os.environ)
    base_env.update(env or {})
    procs = []

    def spawn(job, i, restarts=0, log=None):
        e = dict(base_env)
        if job == "ps" and "DTF_PS_VISIBLE_DEVICES" in e:
            # e.g. "" = a host-memory PS as in the reference (ps_device="/job:ps/cpu:0");
            # by default the PS task keeps the GPU that will hold its HBM-resident shard
            e["HIP_VISIBLE_DEVICES"] = e["DTF_PS_VISIBLE_DEVICES"]
        elif job != "ps" and gpus_per_host:
            e["LOCAL_RANK"] = str(i % gpus_per_host)
        e["DTF_RESTART_COUNT"] = str(restarts)
        log = log or open(os.path.join(workdir, f"{job}{i}.log"), "w")
        cmd = [sys.executable, script, f"--job_name={job}", f"--task_index={i}",
               f"--config={cfg_path}", *extra_args]
        return subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, env=e, cwd=workdir), log

    for job, n in (("ps", num_ps), ("worker", num_workers)):
        for i in range(n):
            p, log = spawn(job, i)
            procs.append([job, i, p, log, 0])
    t0 = time.time()
    rc = {}
    try:
        # supervise: wait for the workers, restarting crashed PS tasks meanwhile
        while True:
            workers_alive = [q for q in procs if q[0] == "worker" and q[2].poll() is None]
            for q in procs:
                job, i, p, log, restarts = q
                if job == "ps" and p.poll() not in (None, 0) and workers_alive and \
                        restarts < max_ps_restarts:
                    _cleanup_shm(p.pid)
                    log.write(f"\n[launcher] ps{i} (pid {p.pid}) exited with {p.returncode}; "
                              f"restarting ({restarts + 1}/{max_ps_restarts})\n")
                    log.flush()
                    q[2], q[3] = spawn(job, i, restarts + 1, log)
                    q[4] = restarts + 1
            if not workers_alive:
                break
            if time.time() - t0 > timeout_s:
                raise subprocess.TimeoutExpired(script, timeout_s)
            time.sleep(0.2)
        for job, i, p, log, _ in procs:
            if job == "worker":
                rc[(job, i)] = p.wait()
        for job, i, p, log, _ in procs:
            if job == "ps":
                try:
                    rc[(job, i)] = p.wait(timeout=grace_s)
                except subprocess.TimeoutExpired:
                    p.terminate()
                    rc[(job, i)] = p.wait(timeout=10)
    finally:
        for job, i, p, log, _ in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            log.close()
    return rc, {f"{j}{i}": os.path.join(workdir, f"{j}{i}.log") for j, i, _, _, _ in procs}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("script")
    ap.add_argument("--num_ps", type=int, default=1)
    ap.add_argument("--num_workers", type=int, default=2)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--max_ps_restarts", type=int, default=0)
    a, rest = ap.parse_known_args()
    codes, logs = launch_local(a.script, a.num_ps, a.num_workers, a.workdir, rest,
                               max_ps_restarts=a.max_ps_restarts)
    print(json.dumps({"exit_codes": {f"{k[0]}{k[1]}": v for k, v in codes.items()},
                      "logs": logs}, indent=2))
