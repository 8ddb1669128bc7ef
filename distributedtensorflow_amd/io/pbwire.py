"""Minimal protobuf wire-format encoder / decoder (no generated code, no TensorFlow).

Used to write TensorFlow's ``SavedModel`` / ``MetaGraphDef`` / ``GraphDef`` messages
(train/saved_model.py) and, in the tests, to read them back independently.  Only what those
messages need: varints, fixed32/64, length-delimited fields, maps as repeated entries.
"""
from __future__ import annotations

import struct


def varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def key(field: int, wire: int) -> bytes:
    return varint((field << 3) | wire)


def f_int(field: int, v: int) -> bytes:
    return key(field, 0) + varint(int(v))


def f_bool(field: int, v: bool) -> bytes:
    return f_int(field, 1 if v else 0)


def f_float(field: int, v: float) -> bytes:
    return key(field, 5) + struct.pack("<f", float(v))


def f_bytes(field: int, b: bytes) -> bytes:
    return key(field, 2) + varint(len(b)) + b


def f_str(field: int, s: str) -> bytes:
    return f_bytes(field, s.encode())


def f_msg(field: int, body: bytes) -> bytes:
    return f_bytes(field, body)


def f_map(field: int, entries, value_enc) -> bytes:
    """map<string, V>: repeated {key = 1, value = 2} entries in key order."""
    return b"".join(f_msg(field, f_str(1, k) + value_enc(2, v))
                    for k, v in sorted(entries.items()))


def f_packed_ints(field: int, vals) -> bytes:
    return f_bytes(field, b"".join(varint(int(v)) for v in vals))


def f_packed_floats(field: int, vals) -> bytes:
    return f_bytes(field, b"".join(struct.pack("<f", float(v)) for v in vals))


# ----------------------------------------------------------------------------- decoding

def _read_varint(b: bytes, i: int):
    shift, v = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v, i
        shift += 7


def parse(b: bytes):
    """{field: [values]}: varints as int, fixed32/64 as raw bytes, length-delimited as bytes."""
    out = {}
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        field, wire = k >> 3, k & 7
        if wire == 0:
            v, i = _read_varint(b, i)
        elif wire == 1:
            v, i = b[i:i + 8], i + 8
        elif wire == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        elif wire == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported wire type {wire}")
        out.setdefault(field, []).append(v)
    return out


def parse_map(entries):
    """Decoded map<string, bytes>: {key: value-bytes} from repeated entry messages."""
    out = {}
    for e in entries:
        d = parse(e)
        out[d[1][0].decode()] = d.get(2, [b""])[0]
    return out


def unpack_varints(b: bytes):
    out, i = [], 0
    while i < len(b):
        v, i = _read_varint(b, i)
        out.append(v if v < (1 << 63) else v - (1 << 64))
    return out


def as_float(raw: bytes) -> float:
    return struct.unpack("<f", raw)[0]
