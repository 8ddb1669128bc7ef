"""TensorBoard event files without TensorFlow.

* :class:`EventFileWriter` — ``events.out.tfevents.<unix>.<host>`` in a log dir, first record
  ``file_version: "brain.Event:2"``; scalar and histogram summaries.  Replaces the reference's
  ``pywrap_tensorflow.EventsWriter`` use in ``logger.TensorBoardOutputFormat``
  (``logger.py:142-165``).  Flushing is batched (every ``flush_secs`` or ``max_queue`` events)
  instead of the reference's per-write ``Flush()``.
* :func:`summary_iterator` / :func:`read_scalars` — the ``tf.train.summary_iterator`` /
  ``logger.read_tb`` reader side.
"""
from __future__ import annotations

import glob
import os
import time

from ..io.native import lib
from ..io.records import tf_record_iterator


class EventFileWriter:
    def __init__(self, logdir: str, filename_suffix: str = "", flush_secs: float = 10.0,
                 max_queue: int = 10):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        self._w = lib().EventsWriter(os.path.join(os.path.abspath(logdir), "events"),
                                     filename_suffix)
        self.flush_secs = flush_secs
        self.max_queue = max_queue
        self._pending = 0
        self._last_flush = time.time()
        self._closed = False

    @property
    def path(self) -> str:
        return self._w.path

    def _after_write(self):
        self._pending += 1
        now = time.time()
        if self._pending >= self.max_queue or now - self._last_flush >= self.flush_secs:
            self.flush()

    def add_scalars(self, kvs: dict, step: int, wall_time: float | None = None):
        items = [(str(k), float(v)) for k, v in kvs.items()]
        self._w.write_event(lib().encode_scalar_event(wall_time or time.time(), int(step), items))
        self._after_write()

    def add_scalar(self, tag: str, value, step: int, wall_time: float | None = None):
        self.add_scalars({tag: value}, step, wall_time)

    def add_histogram(self, tag: str, values, step: int, bins: int = 30,
                      wall_time: float | None = None):
        import numpy as np
        vals = np.asarray(values, dtype=np.float64).reshape(-1).tolist()
        self._w.write_event(lib().encode_histogram_event(wall_time or time.time(), int(step), tag,
                                                         vals, int(bins)))
        self._after_write()

    def flush(self):
        if not self._closed:
            self._w.flush()
        self._pending = 0
        self._last_flush = time.time()

    def close(self):
        if not self._closed:
            self._w.flush()
            self._w.close()
            self._closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


FileWriter = EventFileWriter


def summary_iterator(path: str):
    """Yield parsed events ``{"wall_time","step","file_version","scalars","histograms"}``."""
    parse = lib().parse_event
    for rec in tf_record_iterator(path):
        yield parse(rec)


def event_files(path: str):
    if os.path.isdir(path):
        return sorted(glob.glob(os.path.join(path, "events.*")))
    if os.path.basename(path).startswith("events."):
        return [path]
    raise ValueError(f"expected an events file or a directory containing them: {path}")


def read_scalars(path: str) -> dict:
    """{tag: [(step, value), ...]} over every event file under ``path``."""
    out: dict = {}
    for fn in event_files(path):
        for ev in summary_iterator(fn):
            for tag, val in ev["scalars"]:
                out.setdefault(tag, []).append((ev["step"], val))
    return out
