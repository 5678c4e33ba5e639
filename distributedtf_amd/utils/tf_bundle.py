"""TensorFlow tensor-bundle checkpoints (``model.ckpt.index`` + ``.data-*``): reader and writer.

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

The writer (``write_bundle``) produces the same layout TF 1.x ``Saver`` writes -- one data shard, an index
SSTable (header entry under the empty key, entries sorted by name, restart interval 16, uncompressed blocks with
masked CRC32C trailers, empty metaindex, footer) -- so a member's state can be exported in the reference's
checkpoint format (``ModelBase.export_tf_checkpoint``).  CRC32C runs natively (``ops/csrc/host.hip``, SSE4.2)
with a pure-Python fallback.
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


# ------------------------------------------------------------------------------------------------- writer
_NP2TF = {np.dtype(v): k for k, v in _DTYPES.items()}
_CRC_TABLE = None


def _crc32c_py(data: bytes, crc: int = 0) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        tab = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            tab.append(c)
        _CRC_TABLE = tab
    c = crc ^ 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def crc32c(data: bytes) -> int:
    """CRC32C (Castagnoli): the native SSE4.2 routine of the kernel library when it loads, else Python."""
    try:
        import ctypes
        from .. import ops
        fn = ops.lib().dtf_crc32c
        fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        fn.restype = ctypes.c_uint32
        return int(fn(bytes(data), len(data), 0))
    except Exception:
        return _crc32c_py(bytes(data))


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _put_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _pb_varint(field: int, v: int) -> bytes:
    return _put_varint(field << 3) + _put_varint(v) if v else b""


def _pb_bytes(field: int, b: bytes) -> bytes:
    return _put_varint((field << 3) | 2) + _put_varint(len(b)) + b


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_pb_bytes(2, _pb_varint(1, int(d)) if d else b"") for d in shape)
    msg = _pb_varint(1, dtype) + _pb_bytes(2, dims)
    msg += _pb_varint(4, offset) + _pb_varint(5, size)
    return msg + _put_varint((6 << 3) | 5) + struct.pack("<I", crc)


def _block(entries, restart_interval: int = 16) -> bytes:
    buf, restarts, last = bytearray(), [], b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(buf))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        buf += _put_varint(shared) + _put_varint(len(k) - shared) + _put_varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def _with_trailer(block: bytes) -> bytes:
    return block + b"\x00" + struct.pack("<I", masked_crc32c(block + b"\x00"))


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """Write ``prefix.index`` + ``prefix.data-00000-of-00001`` holding ``tensors`` (name -> array)."""
    names = sorted(tensors)
    data, entries, off = bytearray(), [], 0
    for n in names:
        a = np.asarray(tensors[n])
        if not a.flags.c_contiguous:  # (np.ascontiguousarray would turn scalars into shape (1,))
            a = a.copy()
        dt = _NP2TF.get(a.dtype)
        if dt is None:
            raise ValueError("unsupported dtype %s for %s" % (a.dtype, n))
        raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
        entries.append((n.encode(), _entry_proto(dt, a.shape, off, len(raw), masked_crc32c(raw))))
        data += raw
        off += len(raw)
    header = _pb_varint(1, 1) + _pb_bytes(3, _pb_varint(1, 1))  # num_shards 1, version {producer 1}
    dblock = _with_trailer(_block([(b"", header)] + entries))
    meta = _with_trailer(_block([]))
    last_key = entries[-1][0] if entries else b""
    # LevelDB BytewiseComparator::FindShortSuccessor of the block's last key (what TF's table builder stores)
    for i, byte in enumerate(last_key):
        if byte != 0xFF:
            last_key = last_key[:i] + bytes([byte + 1])
            break
    index = _with_trailer(_block([(last_key, _put_varint(0) + _put_varint(len(dblock) - 5))]))
    meta_off = len(dblock)
    index_off = meta_off + len(meta)
    footer = _put_varint(meta_off) + _put_varint(len(meta) - 5) + _put_varint(index_off) + _put_varint(len(index) - 5)
    footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", _MAGIC)
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    with open(prefix + ".index", "wb") as f:
        f.write(dblock + meta + index + footer)
