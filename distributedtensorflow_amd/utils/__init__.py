"""Small host-side helpers shared by the entry points (bench, launcher tasks)."""
import os

# launch plumbing the bench / launcher set on their own child processes (not configuration)
_PLUMBING = {"DTF_BENCH_LAUNCH", "DTF_STORE_ADDR", "DTF_MAX_RESTARTS", "DTF_RESTART_COUNT"}


def dtf_env():
    """Every ``DTF_*`` variable of this process's environment (launch plumbing excluded): the
    bench JSON records it, so a bench line shows whether it ran the default, tested
    configuration -- an empty dict means every knob at its default."""
    return {k: v for k, v in sorted(os.environ.items())
            if k.startswith("DTF_") and k not in _PLUMBING}
