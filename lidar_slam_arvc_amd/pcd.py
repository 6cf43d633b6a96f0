"""PCD reader for KeyFrame.load_pointcloud (keyframe.py:41-45 -> o3d.io.read_point_cloud).

Reads x, y, z of PCD v0.7 files in DATA ascii / binary / binary_compressed (LZF), the three
encodings Open3D's reader accepts. As Open3D does by default (remove_nan_points=False), NaN/inf
points are kept; they are dropped by filter_radius_height because every comparison with NaN is
false (keyframe.py:92). Returns float32 N x 3. For SIZE 4 binary fields this is the on-disk
precision (Open3D widens it to float64 exactly). SIZE 8 fields and ascii values are ROUNDED to
float32 here, while Open3D keeps them in float64: the device path stores f32 coordinates, so for
such files parity with the reference is unpinned beyond that rounding.
A ``write_pcd`` helper produces test fixtures and synthetic datasets.
"""
from __future__ import annotations

import numpy as np

_NP = {("F", 4): np.float32, ("F", 8): np.float64, ("U", 1): np.uint8, ("U", 2): np.uint16,
       ("U", 4): np.uint32, ("U", 8): np.uint64, ("I", 1): np.int8, ("I", 2): np.int16,
       ("I", 4): np.int32, ("I", 8): np.int64}


def lzf_decompress(src: bytes, out_len: int) -> bytes:
    """LZF (liblzf) decompression, as used by PCL/Open3D for binary_compressed."""
    out = bytearray(out_len)
    ip = op = 0
    n = len(src)
    while ip < n:
        ctrl = src[ip]
        ip += 1
        if ctrl < 32:                     # literal run of ctrl + 1 bytes
            ln = ctrl + 1
            out[op:op + ln] = src[ip:ip + ln]
            ip += ln
            op += ln
        else:                             # back reference
            ln = ctrl >> 5
            ref = op - ((ctrl & 0x1F) << 8) - 1
            if ln == 7:
                ln += src[ip]
                ip += 1
            ref -= src[ip]
            ip += 1
            ln += 2
            if ref < 0:
                raise ValueError("corrupt LZF stream")
            for k in range(ln):           # may overlap: byte by byte
                out[op + k] = out[ref + k]
            op += ln
    if op != out_len:
        raise ValueError(f"LZF size mismatch: {op} != {out_len}")
    return bytes(out)


def read_pcd(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        raw = f.read()
    header = {}
    pos = 0
    while True:
        end = raw.index(b"\n", pos)
        line = raw[pos:end].decode("ascii", "replace").strip()
        pos = end + 1
        if not line or line.startswith("#"):
            continue
        key, _, val = line.partition(" ")
        header[key.upper()] = val.split()
        if key.upper() == "DATA":
            break
    fields = header["FIELDS"]
    sizes = [int(s) for s in header["SIZE"]]
    types = header["TYPE"]
    counts = [int(c) for c in header.get("COUNT", ["1"] * len(fields))]
    npts = int(header.get("POINTS", [0])[0]) or int(header["WIDTH"][0]) * int(header["HEIGHT"][0])
    mode = header["DATA"][0].lower()
    for need in ("x", "y", "z"):
        if need not in fields:
            raise ValueError(f"PCD has no field {need!r}")
    dt = np.dtype([(f"{f}" if c == 1 else f"{f}_", _NP[(t, s)], (c,) if c > 1 else ())
                   for f, s, t, c in zip(fields, sizes, types, counts)])
    body = raw[pos:]
    if mode == "ascii":
        txt = np.loadtxt(body.decode("ascii").splitlines(), ndmin=2)
        cols = []
        off = 0
        for f, c in zip(fields, counts):
            if f in ("x", "y", "z"):
                cols.append((f, off))
            off += c
        idx = dict(cols)
        return np.stack([txt[:npts, idx[a]] for a in "xyz"], axis=1).astype(np.float32)
    if mode == "binary":
        arr = np.frombuffer(body, dtype=dt, count=npts)
    elif mode == "binary_compressed":
        csize, usize = np.frombuffer(body[:8], dtype="<u4")
        data = lzf_decompress(body[8:8 + int(csize)], int(usize))
        # column-major: each field stored contiguously for all points
        arr = np.empty(npts, dtype=dt)
        off = 0
        for name in dt.names:
            sub = dt.fields[name][0]
            nb = sub.itemsize * npts
            arr[name] = np.frombuffer(data[off:off + nb], dtype=sub.base,
                                      count=npts * max(1, int(np.prod(sub.shape)))).reshape(
                arr[name].shape)
            off += nb
    else:
        raise ValueError(f"unsupported PCD DATA mode {mode!r}")
    return np.stack([arr["x"], arr["y"], arr["z"]], axis=1).astype(np.float32)


def write_pcd(path: str, xyz, mode: str = "binary") -> None:
    p = np.ascontiguousarray(np.asarray(xyz, dtype=np.float32))
    head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z\n"
            "SIZE 4 4 4\nTYPE F F F\nCOUNT 1 1 1\n"
            f"WIDTH {len(p)}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {len(p)}\n"
            f"DATA {mode}\n")
    with open(path, "wb") as f:
        f.write(head.encode("ascii"))
        if mode == "ascii":
            np.savetxt(f, p, fmt="%.9g")
        elif mode == "binary":
            f.write(p.tobytes())
        else:
            raise ValueError("write_pcd supports ascii and binary")
