"""TensorBoard scalar event files without the tensorboard package (PPO/main.py:39,101-109, RPO-LSTM/main.py:39).

The reference learners log through ``torch.utils.tensorboard.SummaryWriter("../runs/<run>")``:
``charts/episodic_return``, ``charts/episodic_length`` and ``average/average_reward`` against ``global_step``.
``tensorboard`` is not installed here, so this module writes the same file format itself:

* the file is a TFRecord stream: per record ``uint64 length``, ``uint32 masked_crc32c(length bytes)``, the
  payload, ``uint32 masked_crc32c(payload)`` (little endian; mask ``((c >> 15) | (c << 17)) + 0xa282ead8``);
* every payload is a serialized ``tensorflow.Event`` protobuf: ``wall_time`` (field 1, double), ``step``
  (field 2, int64) and either ``file_version`` (field 3, "brain.Event:2", the first record) or ``summary``
  (field 5) holding ``Summary.value`` (field 1) entries of ``tag`` (field 1, string) and ``simple_value``
  (field 2, float) -- exactly what ``SummaryWriter.add_scalar`` emits for a Python float.

The file is named as SummaryWriter names it, ``events.out.tfevents.<unix time>.<host>.<pid>.0``, inside the run
directory.  ``read_scalars`` parses such a file back (tests/test_learner_cpu.py).
"""
import os
import socket
import struct
import time

_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1   # CRC-32C (Castagnoli), reflected
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1   # int64 two's complement, as protobuf encodes negative int64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, file_version: str = None, scalars=()) -> bytes:
    """One serialized tensorflow.Event: the file-version header or a Summary of (tag, value) scalars."""
    out = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        out += _len_field(3, file_version.encode())
    if scalars:
        summ = b"".join(_len_field(1, _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v)))
                        for tag, v in scalars)
        out += _len_field(5, summ)
    return out


def frame(payload: bytes) -> bytes:
    head = struct.pack("<Q", len(payload))
    return head + struct.pack("<I", masked_crc32c(head)) + payload + struct.pack("<I", masked_crc32c(payload))


class EventWriter:
    """``SummaryWriter(logdir).add_scalar`` for float scalars: one event file in ``logdir``."""

    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        now = time.time()
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(now)}.{socket.gethostname()}.{os.getpid()}.0")
        self._fh = open(self.path, "wb")
        self._fh.write(frame(encode_event(now, 0, file_version="brain.Event:2")))
        self._fh.flush()

    def add_scalar(self, tag: str, value, global_step: int, walltime: float = None):
        self._fh.write(frame(encode_event(time.time() if walltime is None else walltime, global_step,
                                          scalars=[(tag, float(value))])))

    def flush(self):
        self._fh.flush()

    def close(self):
        if not self._fh.closed:
            self._fh.close()


# ------------------------------------------------------------------------------------------ reading back
def _read_varint(b: bytes, i: int):
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return v, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def read_records(path: str):
    """The payloads of a TFRecord file, each CRC checked."""
    with open(path, "rb") as fh:
        data = fh.read()
    i, out = 0, []
    while i < len(data):
        head = data[i:i + 8]
        (n,) = struct.unpack("<Q", head)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        if hc != masked_crc32c(head):
            raise ValueError(f"length CRC mismatch at byte {i}")
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if pc != masked_crc32c(payload):
            raise ValueError(f"payload CRC mismatch at byte {i}")
        out.append(payload)
        i += 16 + n
    return out


def read_scalars(path: str):
    """[(tag, step, value, wall_time)] of every scalar in the file, and the file-version string."""
    version, out = None, []
    for rec in read_records(path):
        wall, step, summ = 0.0, 0, None
        for f, w, v in _fields(rec):
            if f == 1 and w == 1:
                (wall,) = struct.unpack("<d", v)
            elif f == 2 and w == 0:
                step = v - (1 << 64) if v >> 63 else v
            elif f == 3 and w == 2:
                version = v.decode()
            elif f == 5 and w == 2:
                summ = v
        if summ is None:
            continue
        for f, w, val in _fields(summ):
            if f != 1:
                continue
            tag, x = None, None
            for g, w2, y in _fields(val):
                if g == 1:
                    tag = y.decode()
                elif g == 2 and w2 == 5:
                    (x,) = struct.unpack("<f", y)
            out.append((tag, step, x, wall))
    return out, version
