"""Minimal drop-in for the `plyfile` package (not installable here), covering what the
reference uses for scene I/O: `PlyData.read`, `PlyData([PlyElement.describe(arr, 'vertex')])
.write(path)`, `plydata.elements[0][name]`, `plydata.elements[0].properties[i].name` and
`plydata['vertex']` (scene/gaussian_model.py:305-417, scene/dataset_readers.py).

Binary little/big endian and ASCII files with scalar properties are read through numpy
structured dtypes (one `np.frombuffer` per element, no per-row Python work).  List
properties (mesh faces) are parsed for ASCII and binary files too, more slowly.  Writes
binary little endian, as plyfile does by default.
"""
from __future__ import annotations

import numpy as np

__all__ = ["PlyData", "PlyElement", "PlyProperty", "PlyListProperty", "PlyParseError"]

_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2", "ushort": "u2",
    "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4", "float": "f4", "float32": "f4",
    "double": "f8", "float64": "f8",
}
_NAMES = {"i1": "char", "u1": "uchar", "i2": "short", "u2": "ushort", "i4": "int", "u4": "uint", "f4": "float",
          "f8": "double"}


class PlyParseError(Exception):
    pass


class PlyProperty:
    def __init__(self, name, val_dtype):
        self.name = name
        self.val_dtype = val_dtype

    def __repr__(self):
        return f"PlyProperty({self.name!r}, {self.val_dtype!r})"


class PlyListProperty(PlyProperty):
    def __init__(self, name, len_dtype, val_dtype):
        super().__init__(name, val_dtype)
        self.len_dtype = len_dtype


class PlyElement:
    def __init__(self, name, properties, count, data=None, comments=()):
        self.name = name
        self.properties = list(properties)
        self.count = count
        self.data = data
        self.comments = list(comments)

    @staticmethod
    def describe(data, name, comments=()):
        """From a 1-D numpy structured array (plyfile.PlyElement.describe)."""
        if not isinstance(data, np.ndarray) or data.dtype.names is None or data.ndim != 1:
            raise TypeError("describe() needs a one-dimensional structured numpy array")
        props = []
        for n in data.dtype.names:
            dt = data.dtype[n]
            if dt.kind == "O":
                raise TypeError("list properties are not supported by describe() here")
            props.append(PlyProperty(n, dt.str[1:]))
        return PlyElement(name, props, len(data), data, comments)

    def __getitem__(self, key):
        return self.data[key]

    def __setitem__(self, key, value):
        self.data[key] = value

    def __len__(self):
        return self.count

    def _scalar_dtype(self, endian):
        if any(isinstance(p, PlyListProperty) for p in self.properties):
            return None
        return np.dtype([(p.name, endian + p.val_dtype) for p in self.properties])


class PlyData:
    def __init__(self, elements=(), text=False, byte_order="<", comments=(), obj_info=()):
        self.elements = list(elements)
        self.text = text
        self.byte_order = byte_order
        self.comments = list(comments)
        self.obj_info = list(obj_info)

    def __getitem__(self, name):
        for e in self.elements:
            if e.name == name:
                return e
        raise KeyError(name)

    def __contains__(self, name):
        return any(e.name == name for e in self.elements)

    # ---- reading ------------------------------------------------------------------------
    @staticmethod
    def read(stream):
        raw = open(stream, "rb").read() if isinstance(stream, (str, bytes)) or hasattr(stream, "__fspath__") \
            else stream.read()
        end = raw.find(b"end_header")
        if not raw.startswith(b"ply") or end < 0:
            raise PlyParseError("not a PLY file")
        nl = raw.find(b"\n", end)
        header = raw[:end].decode("ascii").splitlines()
        body = raw[nl + 1:]
        fmt, elements, comments, obj_info = None, [], [], []
        for line in header[1:]:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "comment":
                comments.append(line[8:])
            elif tok[0] == "obj_info":
                obj_info.append(line[9:])
            elif tok[0] == "element":
                elements.append(PlyElement(tok[1], [], int(tok[2])))
            elif tok[0] == "property":
                if not elements:
                    raise PlyParseError("property before element")
                if tok[1] == "list":
                    elements[-1].properties.append(PlyListProperty(tok[4], _TYPES[tok[2]], _TYPES[tok[3]]))
                else:
                    if tok[1] not in _TYPES:
                        raise PlyParseError(f"unknown property type {tok[1]}")
                    elements[-1].properties.append(PlyProperty(tok[2], _TYPES[tok[1]]))
        if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
            raise PlyParseError(f"unsupported format {fmt}")
        endian = ">" if fmt == "binary_big_endian" else "<"
        if fmt == "ascii":
            PlyData._read_ascii(elements, body)
        else:
            off = 0
            for e in elements:
                dt = e._scalar_dtype(endian)
                if dt is not None:
                    n = dt.itemsize * e.count
                    if off + n > len(body):
                        raise PlyParseError(f"element {e.name}: file truncated")
                    e.data = np.frombuffer(body, dtype=dt, count=e.count, offset=off).copy()
                    off += n
                else:
                    off = PlyData._read_binary_lists(e, body, off, endian)
        return PlyData(elements, text=fmt == "ascii", byte_order=endian, comments=comments, obj_info=obj_info)

    @staticmethod
    def _read_ascii(elements, body):
        toks = body.split()
        pos = 0
        for e in elements:
            scalar = all(not isinstance(p, PlyListProperty) for p in e.properties)
            if scalar:
                dt = np.dtype([(p.name, p.val_dtype) for p in e.properties])
                k = len(e.properties) * e.count
                vals = np.array(toks[pos:pos + k], dtype=np.float64).reshape(e.count, len(e.properties))
                pos += k
                e.data = np.empty(e.count, dtype=dt)
                for i, p in enumerate(e.properties):
                    e.data[p.name] = vals[:, i].astype(p.val_dtype)
            else:
                dt = np.dtype([(p.name, object if isinstance(p, PlyListProperty) else p.val_dtype)
                               for p in e.properties])
                e.data = np.empty(e.count, dtype=dt)
                for r in range(e.count):
                    for p in e.properties:
                        if isinstance(p, PlyListProperty):
                            n = int(toks[pos])
                            e.data[p.name][r] = np.array(toks[pos + 1:pos + 1 + n], dtype=np.float64).astype(
                                p.val_dtype)
                            pos += 1 + n
                        else:
                            e.data[p.name][r] = float(toks[pos])
                            pos += 1

    @staticmethod
    def _read_binary_lists(e, body, off, endian):
        dt = np.dtype([(p.name, object if isinstance(p, PlyListProperty) else p.val_dtype) for p in e.properties])
        e.data = np.empty(e.count, dtype=dt)
        for r in range(e.count):
            for p in e.properties:
                if isinstance(p, PlyListProperty):
                    lt = np.dtype(endian + p.len_dtype)
                    n = int(np.frombuffer(body, lt, 1, off)[0])
                    off += lt.itemsize
                    vt = np.dtype(endian + p.val_dtype)
                    e.data[p.name][r] = np.frombuffer(body, vt, n, off).copy()
                    off += vt.itemsize * n
                else:
                    vt = np.dtype(endian + p.val_dtype)
                    e.data[p.name][r] = np.frombuffer(body, vt, 1, off)[0]
                    off += vt.itemsize
        return off

    # ---- writing ------------------------------------------------------------------------
    def write(self, stream):
        head = ["ply", "format ascii 1.0" if self.text else "format binary_little_endian 1.0"]
        head += [f"comment {c}" for c in self.comments] + [f"obj_info {c}" for c in self.obj_info]
        for e in self.elements:
            head.append(f"element {e.name} {e.count}")
            head += [f"comment {c}" for c in e.comments]
            for p in e.properties:
                if isinstance(p, PlyListProperty):
                    head.append(f"property list {_NAMES[p.len_dtype]} {_NAMES[p.val_dtype]} {p.name}")
                else:
                    head.append(f"property {_NAMES[p.val_dtype]} {p.name}")
        head.append("end_header")
        out = ("\n".join(head) + "\n").encode("ascii")
        parts = [out]
        for e in self.elements:
            if any(isinstance(p, PlyListProperty) for p in e.properties):
                raise NotImplementedError("writing list properties is not supported here")
            dt = e._scalar_dtype("<")
            arr = np.empty(e.count, dtype=dt)
            for p in e.properties:
                arr[p.name] = e.data[p.name]
            if self.text:
                parts.append(("\n".join(" ".join(repr(v.item()) for v in row) for row in arr) + "\n").encode())
            else:
                parts.append(arr.tobytes())
        data = b"".join(parts)
        if isinstance(stream, (str, bytes)) or hasattr(stream, "__fspath__"):
            with open(stream, "wb") as f:
                f.write(data)
        else:
            stream.write(data)
