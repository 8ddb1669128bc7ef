"""TFRecord files (``tf.io.TFRecordWriter`` / ``tf.compat.v1.io.tf_record_iterator``) on the
native C++ framing code (length + masked CRC32C + payload + masked CRC32C)."""
from __future__ import annotations

from .native import lib


class TFRecordWriter:
    def __init__(self, path: str, append: bool = False):
        self._w = lib().RecordWriter(path, append)

    def write(self, record: bytes):
        self._w.write(bytes(record))

    def flush(self):
        self._w.flush()

    def close(self):
        self._w.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def tf_record_iterator(path: str):
    r = lib().RecordReader(path)
    while True:
        rec = r.next()
        if rec is None:
            return
        yield rec
