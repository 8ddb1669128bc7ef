"""Key/value + text logger with the public API of the reference's ``logger.py``.

Reference: ``logger.py:1-489``.  Same module-level functions (``configure,
logkv, logkv_mean, logkvs, dumpkvs, getkvs, log, debug/info/warn/error, set_level, get_dir,
record_tabular, dump_tabular, ProfileKV, profile, reset, scoped_configure, read_json/read_csv/
read_tb``), same output formats and file names (``log%s.txt``, ``progress%s.json``,
``progress%s.csv``, ``tb%s/``), same env vars (``OPENAI_LOGDIR``, ``OPENAI_LOG_FORMAT``,
``OPENAI_LOG_FORMAT_MPI``, rank from ``PMI_RANK`` / ``OMPI_COMM_WORLD_RANK`` and also torchrun's
``RANK``).  Deliberate differences:

* importing does NOT create a temp dir; the default logger is created lazily (stdout only);
* the TensorBoard sink works with ``dumpkvs()`` (the reference's ``writekvs(kvs, global_step)``
  signature broke it, ``logger.py:157`` vs ``:321``) — it keeps its own step counter when no
  step is given;
* the JSON sink does not mutate the caller's dict;
* TensorBoard events come from the native C++ writer (no TensorFlow).
"""
from __future__ import annotations

import datetime
import json
import os
import sys
import tempfile
import time
from collections import defaultdict

DEBUG, INFO, WARN, ERROR, DISABLED = 10, 20, 30, 40, 50


# ----------------------------------------------------------------------------- sinks

class KVWriter:
    def writekvs(self, kvs, step=None):
        raise NotImplementedError

    def close(self):
        pass


class SeqWriter:
    def writeseq(self, seq):
        raise NotImplementedError


def _fmt_value(v):
    return "%-8.3g" % v if isinstance(v, float) else str(v)


def _clip(s, width=20):
    return s if len(s) <= width + 3 else s[:width] + "..."


class HumanOutputFormat(KVWriter, SeqWriter):
    """ASCII table for key/values, plain lines for ``log()``."""

    def __init__(self, target):
        if isinstance(target, str):
            self.stream, self._owned = open(target, "wt"), True
        else:
            if not hasattr(target, "write"):
                raise TypeError(f"expected a path or a writable stream, got {target!r}")
            self.stream, self._owned = target, False

    def writekvs(self, kvs, step=None):
        if not kvs:
            print("WARNING: tried to write empty key-value dict")
            return
        cells = {_clip(str(k)): _clip(_fmt_value(v)) for k, v in kvs.items()}
        kw = max(len(k) for k in cells)
        vw = max(len(v) for v in cells.values())
        bar = "-" * (kw + vw + 7)
        body = [f"| {k.ljust(kw)} | {cells[k].ljust(vw)} |"
                for k in sorted(cells, key=str.lower)]
        self.stream.write("\n".join([bar, *body, bar]) + "\n")
        self.stream.flush()

    def writeseq(self, seq):
        self.stream.write(" ".join(seq) + "\n")
        self.stream.flush()

    def close(self):
        if self._owned:
            self.stream.close()


class JSONOutputFormat(KVWriter):
    def __init__(self, path):
        self.stream = open(path, "wt")

    def writekvs(self, kvs, step=None):
        row = {}
        for k, v in sorted(kvs.items()):
            if hasattr(v, "dtype"):          # numpy / torch scalars -> float
                v = float(v.tolist() if hasattr(v, "tolist") else v)
            row[k] = v
        self.stream.write(json.dumps(row) + "\n")
        self.stream.flush()

    def close(self):
        self.stream.close()


class CSVOutputFormat(KVWriter):
    """CSV whose header grows when new keys appear (older rows are padded)."""

    def __init__(self, path):
        self.path = path
        self.columns: list[str] = []
        self.rows: list[list[str]] = []
        open(path, "wt").close()

    def writekvs(self, kvs, step=None):
        new = sorted(set(kvs) - set(self.columns))
        if new:
            self.columns.extend(new)
            for r in self.rows:
                r.extend([""] * len(new))
            self._rewrite()
        row = ["" if kvs.get(c) is None else str(kvs.get(c)) for c in self.columns]
        self.rows.append(row)
        with open(self.path, "at") as fh:
            fh.write(",".join(row) + "\n")

    def _rewrite(self):
        with open(self.path, "wt") as fh:
            fh.write(",".join(self.columns) + "\n")
            for r in self.rows:
                fh.write(",".join(r) + "\n")

    def close(self):
        pass


class TensorBoardOutputFormat(KVWriter):
    """Scalars to ``<dir>/events.out.tfevents.*`` (native writer).  ``writekvs(kvs, step)``
    accepts the reference's keyword ``global_step`` too."""

    def __init__(self, dir):  # noqa: A002 (reference signature)
        from .events import EventFileWriter
        os.makedirs(dir, exist_ok=True)
        self.dir = dir
        self.step = 1
        self.writer = EventFileWriter(dir, flush_secs=5.0, max_queue=1)

    def writekvs(self, kvs, step=None, global_step=None):
        s = global_step if global_step is not None else step
        if s is None:
            s = self.step
            self.step += 1
        vals = {}
        for k, v in kvs.items():
            try:
                vals[k] = float(v)
            except (TypeError, ValueError):
                continue
        self.writer.add_scalars(vals, int(s))

    def close(self):
        if self.writer is not None:
            self.writer.close()
            self.writer = None


def make_output_format(format, ev_dir, log_suffix=""):  # noqa: A002
    os.makedirs(ev_dir, exist_ok=True)
    if format == "stdout":
        return HumanOutputFormat(sys.stdout)
    if format == "log":
        return HumanOutputFormat(os.path.join(ev_dir, f"log{log_suffix}.txt"))
    if format == "json":
        return JSONOutputFormat(os.path.join(ev_dir, f"progress{log_suffix}.json"))
    if format == "csv":
        return CSVOutputFormat(os.path.join(ev_dir, f"progress{log_suffix}.csv"))
    if format == "tensorboard":
        return TensorBoardOutputFormat(os.path.join(ev_dir, f"tb{log_suffix}"))
    raise ValueError(f"Unknown format specified: {format}")


# ----------------------------------------------------------------------------- backend

class Logger:
    DEFAULT = None
    CURRENT = None

    def __init__(self, dir, output_formats):  # noqa: A002
        self.name2val = defaultdict(float)
        self.name2cnt = defaultdict(int)
        self.level = INFO
        self.dir = dir
        self.output_formats = list(output_formats)
        self.step = None

    def logkv(self, key, val):
        self.name2val[key] = val

    def logkv_mean(self, key, val):
        if val is None:
            self.name2val[key] = None
            return
        n = self.name2cnt[key]
        old = self.name2val[key] or 0.0
        self.name2val[key] = old * n / (n + 1) + val / (n + 1)
        self.name2cnt[key] = n + 1

    def dumpkvs(self, step=None):
        if self.level == DISABLED:
            return
        snapshot = dict(self.name2val)
        for f in self.output_formats:
            if isinstance(f, KVWriter):
                f.writekvs(snapshot, step if step is not None else self.step)
        self.name2val.clear()
        self.name2cnt.clear()

    def log(self, *args, level=INFO):
        if self.level <= level:
            for f in self.output_formats:
                if isinstance(f, SeqWriter):
                    f.writeseq([str(a) for a in args])

    def set_level(self, level):
        self.level = level

    def get_dir(self):
        return self.dir

    def close(self):
        for f in self.output_formats:
            f.close()


def _rank_from_env() -> int:
    for var in ("PMI_RANK", "OMPI_COMM_WORLD_RANK", "RANK"):
        if var in os.environ:
            try:
                return int(os.environ[var])
            except ValueError:
                pass
    return 0


def configure(dir=None, format_strs=None):  # noqa: A002
    if dir is None:
        dir = os.getenv("OPENAI_LOGDIR")
    if dir is None:
        stamp = datetime.datetime.now().strftime("openai-%Y-%m-%d-%H-%M-%S-%f")
        dir = os.path.join(tempfile.gettempdir(), stamp)
    os.makedirs(dir, exist_ok=True)
    rank = _rank_from_env()
    suffix = f"-rank{rank:03d}" if rank > 0 else ""
    if format_strs is None:
        env = "OPENAI_LOG_FORMAT" if rank == 0 else "OPENAI_LOG_FORMAT_MPI"
        default = "stdout,log,csv" if rank == 0 else "log"
        format_strs = os.getenv(env, default).split(",")
    formats = [make_output_format(f, dir, suffix) for f in format_strs if f]
    Logger.CURRENT = Logger(dir, formats)
    log(f"Logging to {dir}")


def _current() -> Logger:
    if Logger.CURRENT is None:
        if "OPENAI_LOG_FORMAT" in os.environ:
            configure()
        else:
            Logger.CURRENT = Logger(None, [HumanOutputFormat(sys.stdout)])
        Logger.DEFAULT = Logger.CURRENT
    return Logger.CURRENT


def reset():
    cur = Logger.CURRENT
    if cur is not None and cur is not Logger.DEFAULT:
        cur.close()
        Logger.CURRENT = Logger.DEFAULT
        log("Reset logger")


class scoped_configure:  # noqa: N801 (reference name)
    def __init__(self, dir=None, format_strs=None):  # noqa: A002
        self.dir, self.format_strs, self.prev = dir, format_strs, None

    def __enter__(self):
        self.prev = Logger.CURRENT
        configure(self.dir, self.format_strs)
        return Logger.CURRENT

    def __exit__(self, *exc):
        Logger.CURRENT.close()
        Logger.CURRENT = self.prev


# ----------------------------------------------------------------------------- module API

def logkv(key, val):
    _current().logkv(key, val)


def logkv_mean(key, val):
    _current().logkv_mean(key, val)


def logkvs(d):
    for k, v in d.items():
        logkv(k, v)


def dumpkvs(step=None):
    _current().dumpkvs(step)


def getkvs():
    return _current().name2val


def log(*args, level=INFO):
    _current().log(*args, level=level)


def debug(*args):
    log(*args, level=DEBUG)


def info(*args):
    log(*args, level=INFO)


def warn(*args):
    log(*args, level=WARN)


def error(*args):
    log(*args, level=ERROR)


def set_level(level):
    _current().set_level(level)


def get_dir():
    return _current().get_dir()


record_tabular = logkv
dump_tabular = dumpkvs


class ProfileKV:
    """``with ProfileKV("x"):`` accumulates wall seconds into key ``wait_x``."""

    def __init__(self, n):
        self.n = "wait_" + n

    def __enter__(self):
        self.t1 = time.time()

    def __exit__(self, *exc):
        _current().name2val[self.n] += time.time() - self.t1


def profile(n):
    def deco(fn):
        def wrapped(*a, **k):
            with ProfileKV(n):
                return fn(*a, **k)
        wrapped.__name__ = getattr(fn, "__name__", "wrapped")
        return wrapped
    return deco


# ----------------------------------------------------------------------------- readers

def read_json(fname):
    import pandas
    with open(fname, "rt") as fh:
        return pandas.DataFrame([json.loads(line) for line in fh if line.strip()])


def read_csv(fname):
    import pandas
    return pandas.read_csv(fname, index_col=None, comment="#")


def read_tb(path):
    """step x tag DataFrame from events files (native reader; no TensorFlow)."""
    import numpy as np
    import pandas

    from .events import read_scalars
    series = read_scalars(path)
    tags = sorted(series)
    maxstep = max((s for pairs in series.values() for s, _ in pairs if s > 0), default=0)
    data = np.full((maxstep, len(tags)), np.nan)
    for j, tag in enumerate(tags):
        for step, val in series[tag]:
            if step > 0:
                data[step - 1, j] = val
    return pandas.DataFrame(data, columns=tags)
