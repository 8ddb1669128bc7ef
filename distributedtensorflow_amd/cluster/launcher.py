"""Local cluster launcher: start every task of a cluster as its own process and keep it alive.

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


class _Task:
    def __init__(self, job, index, spawn):
        self.job, self.index, self._spawn = job, index, spawn
        self.restarts = 0
        self.log = None
        self.proc = None
        self.done = False           # exited 0
        self.start()

    def start(self):
        self.proc, self.log = self._spawn(self.job, self.index, self.restarts, self.log)

    @property
    def name(self):
        return f"{self.job}{self.index}"


def _dump_stacks(tasks):
    """Ask every live task for a Python stack dump into its log (SIGUSR1: the entry scripts
    register faulthandler for it) before a timed-out or failed job is torn down, so a hang is
    diagnosable from the logs alone."""
    import signal
    live = [t for t in tasks if t.proc.poll() is None]
    for t in live:
        try:
            os.kill(t.proc.pid, signal.SIGUSR1)
        except OSError:
            pass
    if live:
        time.sleep(1.0)


def log_tails(tasks, chars=6000):
    """{task name: last ``chars`` characters of its log} (flushes the launcher's own notes)."""
    out = {}
    for t in tasks:
        try:
            t.log.flush()
            with open(t.log.name, errors="replace") as f:
                out[t.name] = f.read()[-chars:]
        except (OSError, ValueError):
            out[t.name] = "<log unreadable>"
    return out


class LaunchTimeout(subprocess.TimeoutExpired):
    """The job did not finish within ``timeout_s``.  Unlike a bare TimeoutExpired its message
    carries every task's log tail -- including the SIGUSR1 stack dumps of the tasks that were
    still alive -- so a hang on a remote box is diagnosable from the failure alone."""

    def __init__(self, cmd, timeout, tails, alive):
        super().__init__(cmd, timeout)
        self.tails, self.alive = tails, alive

    def __str__(self):
        parts = [super().__str__(), f"tasks still alive at the deadline: {self.alive}"]
        for name, text in self.tails.items():
            parts.append(f"===== {name} (log tail) =====\n{text}")
        return "\n".join(parts)


def _stop_others(tasks, failed, rc, grace_s=10.0):
    """A task failed for good: SIGTERM the other live tasks, SIGKILL whatever is still alive
    after ``grace_s`` (a task stuck in a device-side wait may ignore the first signal).  Their
    stacks are dumped into their logs first: where the survivors were is what a failure report
    needs."""
    live = [x for x in tasks if x is not failed and x.proc.poll() is None]
    _dump_stacks(live)
    for x in live:
        x.log.write(f"\n[launcher] {failed.name} failed for good (exit {rc}); stopping "
                    f"{x.name}\n")
        x.log.flush()
        x.final = True          # stopped on purpose: never mistaken for a crash to restart
        x.proc.terminate()
    t0 = time.time()
    while time.time() - t0 < grace_s and any(x.proc.poll() is None for x in live):
        time.sleep(0.1)
    for x in live:
        if x.proc.poll() is None:
            x.proc.kill()
            x.proc.wait()


def _supervise(tasks, store, is_worker, max_restarts, timeout_s, script, restart_alone=False,
               needs_all=False):
    """Wait for the worker tasks, restarting failed tasks meanwhile.

    A task that exits non-zero while the job runs is restarted as a FRESH process (never a
    re-exec of a process that touched the GPU) after the cluster epoch is bumped, so every
    survivor re-forms its process group with it (cluster/rendezvous.py).  Exit code
    ``REJOIN_EXIT_CODE`` is a parameter-server task leaving voluntarily for the new epoch: it is
    restarted without counting against ``max_restarts``.  Once a worker finished cleanly the job
    is ending and failures are no longer recovered.  ``restart_alone``: a collective world
    restarts a failed rank even when no other rank is alive (a one-rank world, or every rank
    died): the restarted ranks resume from the chief's latest checkpoint.

    A task that fails FOR GOOD while the job is not ending (restarts used up, or nobody left to
    re-form the cluster with) ends the job at once when the others cannot finish without it -- a
    parameter-server task, any rank of a collective world (``restart_alone``), any worker of a
    synchronous job (``needs_all``): they could only wait for it until their own timeouts, so
    they are stopped (stacks dumped into their logs first) and the exit codes report the failure.
    A worker of an asynchronous parameter-server job is not needed by the others (between-graph
    training: the chief and the other workers keep training, as in TF1), so its failure is
    logged and the job goes on.  At ``timeout_s`` every live task's stack is dumped and
    :class:`LaunchTimeout` is raised with all log tails in its message."""
    from .rendezvous import bump_epoch
    from .server import Server
    t0 = time.time()
    used = 0
    while True:
        ending = any(t.done for t in tasks if is_worker(t))
        for t in tasks:
            rc = t.proc.poll()
            if rc is None or t.done or getattr(t, "final", False):
                continue
            if rc == 0:
                t.done = True
                continue
            workers_alive = any(x.proc.poll() is None for x in tasks if is_worker(x))
            voluntary = rc == Server.REJOIN_EXIT_CODE
            if ending or not (workers_alive or not is_worker(t) or restart_alone) or \
                    (not voluntary and used >= max_restarts):
                t.final = True
                if not ending:
                    fatal = needs_all or restart_alone or not is_worker(t)
                    t.log.write(f"\n[launcher] {t.name} (pid {t.proc.pid}) exited with {rc} "
                                f"and is not restarted ({used}/{max_restarts} restarts used)"
                                + ("" if fatal else "; the other tasks continue (asynchronous "
                                   "training does not need this worker)") + "\n")
                    t.log.flush()
                    if fatal:
                        _stop_others(tasks, t, rc)
                continue
            if not voluntary:
                used += 1
                epoch = bump_epoch(store)
            else:
                epoch = None
            _cleanup_shm(t.proc.pid)
            t.log.write(f"\n[launcher] {t.name} (pid {t.proc.pid}) exited with {rc}; "
                        + (f"restarting ({used}/{max_restarts}), cluster epoch {epoch}\n"
                           if not voluntary else "rejoining the new cluster epoch\n"))
            t.log.flush()
            t.restarts += 1
            t.start()
        workers = [t for t in tasks if is_worker(t)]
        # every worker exited, and each one either finished or failed for good (a failed task
        # that is restarted is running again by now)
        if all(t.proc.poll() is not None and (t.done or getattr(t, "final", False))
               for t in workers):
            return
        if time.time() - t0 > timeout_s:
            alive = [t.name for t in tasks if t.proc.poll() is None]
            _dump_stacks(tasks)
            raise LaunchTimeout(script, timeout_s, log_tails(tasks), alive)
        time.sleep(0.1)


def launch_local(script, num_ps=1, num_workers=2, workdir=None, extra_args=(), env=None,
                 timeout_s=600, grace_s=30, gpus_per_host=None, max_ps_restarts=0,
                 max_restarts=0, sync=False):
    """Start a PS/worker cluster of ``script`` on this host and supervise it.

    ``sync``: the workers train synchronously (SyncReplicas: every step waits for all of them),
    so a worker that fails for good ends the job; by default (asynchronous between-graph
    training) only a failed PS task does, and the other workers carry on.

    The launcher hosts the cluster's rendezvous store (at the chief's ``config.json`` address),
    so any task -- the chief included -- may die: up to ``max_restarts`` failed tasks (or
    ``max_ps_restarts``, the round-2 name) are restarted as fresh processes in a new cluster
    epoch; survivors re-form the cluster with them and the chief re-seeds the parameter servers
    from the latest checkpoint (MonitoredTrainingSession)."""
    from .rendezvous import connect
    from .spec import Config
    max_restarts = max(int(max_restarts), int(max_ps_restarts))
    workdir = os.path.abspath(workdir or os.getcwd())
    script = os.path.abspath(script)          # tasks run with cwd=workdir
    os.makedirs(workdir, exist_ok=True)
    cfg_path = os.path.join(workdir, "config.json")
    write_config(cfg_path, num_ps, num_workers)
    host, port = Config(cfg_path).cluster_spec().rendezvous_address()
    store = connect(timeout_s=60, host=host, port=port, is_master=True)
    base_env = dict(os.environ)
    base_env.update(env or {})
    base_env["DTF_STORE_ADDR"] = f"{host}:{port}"
    base_env["DTF_MAX_RESTARTS"] = str(max_restarts)

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

    tasks = [_Task(job, i, spawn) for job, n in (("ps", num_ps), ("worker", num_workers))
             for i in range(n)]
    rc = {}
    try:
        _supervise(tasks, store, lambda t: t.job == "worker", max_restarts, timeout_s, script,
                   needs_all=sync)
        for t in tasks:
            if t.job == "worker":
                rc[(t.job, t.index)] = t.proc.wait()
        for t in tasks:
            if t.job == "ps":
                try:
                    rc[(t.job, t.index)] = t.proc.wait(timeout=grace_s)
                except subprocess.TimeoutExpired:
                    t.proc.terminate()
                    rc[(t.job, t.index)] = t.proc.wait(timeout=10)
    finally:
        for t in tasks:
            if t.proc.poll() is None:
                t.proc.kill()
                t.proc.wait()
            t.log.close()
    return rc, {t.name: os.path.join(workdir, f"{t.name}.log") for t in tasks}


def launch_collective(script, nproc, workdir=None, extra_args=(), env=None, timeout_s=600,
                      max_restarts=0):
    """torchrun-style launch of a synchronous world (Mirrored / MultiWorkerMirrored / colocated
    PS): ``nproc`` ranks with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* set, the rendezvous store
    hosted HERE.  A rank that dies is restarted alone (up to ``max_restarts``) in a new cluster
    epoch; the surviving ranks re-form the world with it in-process and continue from the
    chief's latest checkpoint (unlike torchrun, which restarts every rank)."""
    from .rendezvous import connect
    workdir = os.path.abspath(workdir or os.getcwd())
    os.makedirs(workdir, exist_ok=True)
    port = free_ports(1)[0]
    store = connect(timeout_s=60, host="127.0.0.1", port=port, is_master=True)
    base_env = dict(os.environ)
    base_env.update(env or {})
    base_env.update({"WORLD_SIZE": str(nproc), "LOCAL_WORLD_SIZE": str(nproc),
                     "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                     "DTF_STORE_ADDR": f"127.0.0.1:{port}", "DTF_MAX_RESTARTS": str(max_restarts)})

    def spawn(job, r, restarts=0, log=None):
        e = dict(base_env, RANK=str(r), LOCAL_RANK=str(r), DTF_RESTART_COUNT=str(restarts))
        log = log or open(os.path.join(workdir, f"rank{r}.log"), "w")
        return subprocess.Popen([sys.executable, os.path.abspath(script), *extra_args],
                                stdout=log, stderr=subprocess.STDOUT, env=e, cwd=workdir), log

    tasks = [_Task("rank", r, spawn) for r in range(nproc)]
    rc = {}
    try:
        _supervise(tasks, store, lambda t: True, max_restarts, timeout_s, script,
                   restart_alone=True)
        for t in tasks:
            rc[t.index] = t.proc.wait()
    finally:
        for t in tasks:
            if t.proc.poll() is None:
                t.proc.kill()
                t.proc.wait()
            t.log.close()
    return rc, {t.name: os.path.join(workdir, f"{t.name}.log") for t in tasks}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("script")
    ap.add_argument("--num_ps", type=int, default=1)
    ap.add_argument("--num_workers", type=int, default=2)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--max_restarts", "--max_ps_restarts", type=int, default=0)
    ap.add_argument("--sync", action="store_true",
                    help="synchronous workers: a worker failing for good ends the job")
    a, rest = ap.parse_known_args()
    codes, logs = launch_local(a.script, a.num_ps, a.num_workers, a.workdir, rest,
                               max_restarts=a.max_restarts, sync=a.sync)
    print(json.dumps({"exit_codes": {f"{k[0]}{k[1]}": v for k, v in codes.items()},
                      "logs": logs}, indent=2))
