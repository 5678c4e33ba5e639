"""Read-only parser for TensorFlow tensor-bundle checkpoints (``model.ckpt.index`` + ``.data-*``).

Used by the golden-fixture tests (reference ``official/utils/testing/reference_data``,
SURVEY §4): the reference's only numerics fixtures are TF 1.x checkpoints, and
TensorFlow is not available here.  Nothing in the files is executed: the index
is a LevelDB-format SSTable whose values are ``BundleEntryProto`` messages, which
are decoded field by field (varints / length-delimited), and tensor bytes are
read with ``numpy.frombuffer``.

Format notes (public LevelDB / TF tensor_bundle specs):
  footer (last 48 bytes) = metaindex BlockHandle, index BlockHandle, padding, magic 0xdb4775248b80fb57;
  block = entries (shared varint, non-shared varint, value-len varint, key delta, value) + restarts + trailer
  (1-byte compression type, 4-byte crc); BundleEntryProto: 1 dtype, 2 shape{2 dim{1 size}}, 3 shard_id,
  4 offset, 5 size, 6 crc32c.
"""

from __future__ import annotations

import os
import struct
from typing import Dict, Tuple

import numpy as np

_MAGIC = 0xDB4775248B80FB57
# tensorflow DataType enum -> numpy
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
           10: np.bool_, 14: np.uint16, 19: np.float16}


def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _block_entries(data: bytes, offset: int, size: int):
    block = data[offset:offset + size]
    trailer = data[offset + size:offset + size + 5]
    if trailer and trailer[0] != 0:
        raise ValueError("compressed SSTable blocks are not supported")
    n_restarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * n_restarts
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(block, pos)
        nonshared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        yield key, block[pos:pos + vlen]
        pos += vlen


def _handle(buf: bytes, pos: int) -> Tuple[int, int, int]:
    off, pos = _varint(buf, pos)
    size, pos = _varint(buf, pos)
    return off, size, pos


def _fields(msg: bytes):
    pos = 0
    while pos < len(msg):
        tag, pos = _varint(msg, pos)
        field, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _varint(msg, pos)
        elif wt == 1:
            v = msg[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(msg, pos)
            v = msg[pos:pos + ln]
            pos += ln
        elif wt == 5:
            v = msg[pos:pos + 4]
            pos += 4
        else:
            raise ValueError("unsupported protobuf wire type %d" % wt)
        yield field, v


def _entry(msg: bytes) -> dict:
    e = {"dtype": 1, "shape": [], "shard_id": 0, "offset": 0, "size": 0}
    for f, v in _fields(msg):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            for f2, dim in _fields(v):
                if f2 == 2:
                    size = 0
                    for f3, v3 in _fields(dim):
                        if f3 == 1:
                            size = v3
                    e["shape"].append(size)
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
    return e


def read_index(prefix: str) -> Dict[str, dict]:
    with open(prefix + ".index", "rb") as f:
        data = f.read()
    magic = struct.unpack_from("<Q", data, len(data) - 8)[0]
    if magic != _MAGIC:
        raise ValueError("%s.index is not a TF tensor-bundle index" % prefix)
    footer = data[len(data) - 48:]
    _, _, pos = _handle(footer, 0)
    idx_off, idx_size, _ = _handle(footer, pos)
    out = {}
    for _, hval in _block_entries(data, idx_off, idx_size):
        boff, bsize, _ = _handle(hval, 0)
        for key, val in _block_entries(data, boff, bsize):
            if key == b"":
                continue  # BundleHeaderProto
            out[key.decode()] = _entry(val)
    return out


def load_bundle(prefix: str) -> Dict[str, np.ndarray]:
    """All tensors of a checkpoint prefix (e.g. ``.../model.ckpt``) as numpy arrays."""
    entries = read_index(prefix)
    shards = {}
    out = {}
    d = os.path.dirname(prefix) or "."
    base = os.path.basename(prefix)
    for name, e in entries.items():
        sid = e["shard_id"]
        if sid not in shards:
            cands = [f for f in os.listdir(d) if f.startswith(base + ".data-%05d-of-" % sid)]
            if not cands:
                raise FileNotFoundError("missing data shard %d for %s" % (sid, prefix))
            with open(os.path.join(d, cands[0]), "rb") as f:
                shards[sid] = f.read()
        dt = _DTYPES.get(e["dtype"])
        if dt is None:
            raise ValueError("unsupported dtype %d for %s" % (e["dtype"], name))
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        out[name] = np.frombuffer(raw, dtype=dt).reshape(e["shape"]).copy()
    return out
