"""A task script for tests/test_launcher.py: takes the launcher's flags and misbehaves as told by
``LAUNCHER_TASK_MODE`` (no GPU, no process group)."""
import argparse
import faulthandler
import os
import signal
import sys
import time


def stalled_wait():
    # a recognisable frame for the stack dump
    time.sleep(600)


def main():
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--job_name")
    ap.add_argument("--task_index", type=int)
    ap.add_argument("--config")
    a, _ = ap.parse_known_args()
    mode = os.environ.get("LAUNCHER_TASK_MODE", "ok")
    print(f"task {a.job_name}:{a.task_index} mode {mode}", flush=True)
    if mode == "hang" and a.job_name == "worker" and a.task_index == 1:
        stalled_wait()
    if mode == "worker_fail":
        # asynchronous job: worker 1 dies at once, the chief keeps training and finishes, the PS
        # returns from join() once the chief is done
        done = os.path.join(os.environ["LAUNCHER_TASK_DIR"], "done_worker0")
        if a.job_name == "worker" and a.task_index == 1:
            sys.exit(5)
        if a.job_name == "worker":
            time.sleep(2.0)
            open(done, "w").close()
            return 0
        t0 = time.time()
        while not os.path.exists(done) and time.time() - t0 < 30:
            time.sleep(0.05)
        return 0
    if mode == "ps_fail":
        ready = os.environ.get("LAUNCHER_TASK_DIR")
        if a.job_name == "ps":
            # fail only once both workers can dump their stacks (SIGUSR1 handler installed)
            t0 = time.time()
            while ready and time.time() - t0 < 30 and not all(
                    os.path.exists(os.path.join(ready, f"ready_worker{i}")) for i in (0, 1)):
                time.sleep(0.05)
            sys.exit(3)
        if ready:
            open(os.path.join(ready, f"ready_{a.job_name}{a.task_index}"), "w").close()
        stalled_wait()
    return 0


if __name__ == "__main__":
    sys.exit(main())
