"""NFIO: a tiny named-array container shared by the workload generator, the
CPU oracle (oracle/nf_oracle.c), the reference harness (oracle/ref_harness.cpp)
and the tests.

Layout (little endian):
    magic  b"NFIO0001"
    u32    count
    repeat count times:
        char[24] name (NUL padded)
        u32      dtype code (see _CODES)
        u32      ndim (<= 4)
        u64[4]   shape (unused dims = 1)
        u64      nbytes
        bytes    data (C order), padded to 8 bytes
"""
import struct

import numpy as np

MAGIC = b"NFIO0001"
_CODES = {
    np.dtype(np.int8): 1, np.dtype(np.uint8): 2, np.dtype(np.int16): 3,
    np.dtype(np.uint16): 4, np.dtype(np.int32): 5, np.dtype(np.uint32): 6,
    np.dtype(np.int64): 7, np.dtype(np.uint64): 8, np.dtype(np.float32): 9,
    np.dtype(np.float64): 10,
}
_DTYPES = {v: k for k, v in _CODES.items()}


def write(path, arrays):
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<I", len(arrays)))
        for name, a in arrays.items():
            a = np.ascontiguousarray(a)
            if a.dtype.fields is not None:   # structured records travel as raw bytes
                a = a.view(np.uint8).reshape(a.shape + (a.dtype.itemsize,))
            if a.dtype not in _CODES:
                raise TypeError(f"{name}: unsupported dtype {a.dtype}")
            if a.ndim > 4:
                raise ValueError(f"{name}: ndim > 4")
            nb = name.encode()
            if len(nb) >= 24:
                raise ValueError(f"name too long: {name}")
            shape = list(a.shape) + [1] * (4 - a.ndim)
            f.write(nb.ljust(24, b"\0"))
            f.write(struct.pack("<II4QQ", _CODES[a.dtype], a.ndim, *shape, a.nbytes))
            f.write(a.tobytes())
            pad = (-a.nbytes) % 8
            if pad:
                f.write(b"\0" * pad)


def read(path):
    out = {}
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:8] != MAGIC:
        raise ValueError(f"{path}: bad magic")
    (count,) = struct.unpack_from("<I", buf, 8)
    off = 12
    for _ in range(count):
        name = buf[off:off + 24].rstrip(b"\0").decode()
        off += 24
        code, ndim, s0, s1, s2, s3, nbytes = struct.unpack_from("<II4QQ", buf, off)
        off += struct.calcsize("<II4QQ")
        shape = (s0, s1, s2, s3)[:ndim]
        a = np.frombuffer(buf, dtype=_DTYPES[code], count=nbytes // _DTYPES[code].itemsize,
                          offset=off).reshape(shape).copy()
        out[name] = a
        off += nbytes + ((-nbytes) % 8)
    return out
