"""Minimal TensorBoard event-file writer with the ``tensorboard_logger`` API.

The reference logs through ``tensorboard_logger.Logger(logdir, flush_secs=2)`` and
``log_value(tag, value, step)`` (main_supcon.py:376-379, 327-333, 393-395). That package
is not installed here, so this module writes the TFRecord/``Event`` protobuf format
directly (hand-encoded protobuf + masked CRC32C framing). Files are readable by any
TensorBoard. A JSONL mirror (``scalars.jsonl``) is written next to it for tooling.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

_CRC_TABLE = []


def _make_table():
    poly = 0x82F63B78
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        _CRC_TABLE.append(c)


_make_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int = 0, file_version: str | None = None,
                 tag: str | None = None, value: float | None = None) -> bytes:
    ev = _varint((1 << 3) | 1) + struct.pack("<d", wall_time)
    ev += _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        ev += _field_bytes(3, file_version.encode())
    if tag is not None:
        val = _field_bytes(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
        summary = _field_bytes(1, val)
        ev += _field_bytes(5, summary)
    return ev


def frame(record: bytes) -> bytes:
    header = struct.pack("<Q", len(record))
    return header + struct.pack("<I", masked_crc(header)) + record + struct.pack("<I", masked_crc(record))


def read_events(path: str):
    """Parse a file written by :class:`Logger` back into (step, tag, value) tuples (tests)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (hc,) = struct.unpack_from("<I", data, i + 8)
        assert hc == masked_crc(data[i:i + 8]), "header crc"
        rec = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack_from("<I", data, i + 12 + n)
        assert dc == masked_crc(rec), "data crc"
        i += 16 + n
        out.append(_decode_event(rec))
    return out


def _read_varint(b: bytes, i: int):
    shift = 0
    v = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << shift
        shift += 7
        if not x & 0x80:
            return v, i


def _decode_fields(b: bytes):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = struct.unpack_from("<d", b, i)[0]
            i += 8
        elif wt == 5:
            v = struct.unpack_from("<f", b, i)[0]
            i += 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(wt)
        yield num, v


def _decode_event(rec: bytes):
    step, tag, value = 0, None, None
    for num, v in _decode_fields(rec):
        if num == 2:
            step = v
        elif num == 5:
            for n2, val in _decode_fields(v):
                if n2 == 1:
                    for n3, x in _decode_fields(val):
                        if n3 == 1:
                            tag = x.decode()
                        elif n3 == 2:
                            value = x
    return step, tag, value


class Logger:
    """Drop-in for ``tensorboard_logger.Logger``."""

    def __init__(self, logdir: str, flush_secs: float = 2.0):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        self.flush_secs = flush_secs
        fname = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
        self.path = os.path.join(logdir, fname)
        self._f = open(self.path, "ab")
        self._jsonl = open(os.path.join(logdir, "scalars.jsonl"), "a")
        self._last_flush = time.time()
        self._f.write(frame(encode_event(time.time(), 0, file_version="brain.Event:2")))

    def log_value(self, name: str, value, step: int | None = None):
        value = float(value)
        step = 0 if step is None else int(step)
        self._f.write(frame(encode_event(time.time(), step, tag=name, value=value)))
        self._jsonl.write(json.dumps({"tag": name, "value": value, "step": step}) + "\n")
        if time.time() - self._last_flush >= self.flush_secs:
            self.flush()

    def flush(self):
        self._f.flush()
        self._jsonl.flush()
        self._last_flush = time.time()

    def close(self):
        self.flush()
        self._f.close()
        self._jsonl.close()
