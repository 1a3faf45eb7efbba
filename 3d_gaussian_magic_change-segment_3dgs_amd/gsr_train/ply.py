"""PLY IO of Gaussian models (scene/gaussian_model.py:187-262, the merge of
visualizer.py:196-226) without plyfile.

The host side only parses / formats the header and moves the vertex block as one
float32 matrix (numpy views of the file, one H2D or D2H copy); the row <-> arena
transposition runs on the GPU (gsr_ply_rows_to_arena / gsr_arena_to_ply_rows,
include/gsr_train.h).  Files are what plyfile writes for the reference's
save_ply: `format binary_little_endian 1.0`, one `vertex` element of `float`
properties named by construct_list_of_attributes().  Reading also accepts
big-endian and ascii files and non-float32 properties (converted on the host).
"""
import ctypes

import numpy as np
import torch

from . import _C

_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}

_lib = _C._lib
_lib.gsr_ply_rows_to_arena.restype = ctypes.c_int
_lib.gsr_ply_rows_to_arena.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p]
_lib.gsr_arena_to_ply_rows.restype = ctypes.c_int
_lib.gsr_arena_to_ply_rows.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_void_p]


def attribute_names(M, C):
    """construct_list_of_attributes (gaussian_model.py:187-205) for M SH coefficients
    per channel and C segment classes."""
    names = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)]
    names += [f"f_rest_{i}" for i in range(3 * (M - 1))]
    names += ["opacity"] + [f"segment_{i}" for i in range(C)]
    names += [f"scale_{i}" for i in range(3)] + [f"rot_{i}" for i in range(4)]
    return names


def arena_columns(names, M, C):
    """Row column of every arena float of one Gaussian (arena order), from the
    property names.  Raises KeyError for a missing attribute like the reference."""
    idx = {n: i for i, n in enumerate(names)}

    def need(n):
        if n not in idx:
            raise KeyError(f"PLY vertex element has no property {n!r}")
        return idx[n]

    n_rest = sum(1 for n in names if n.startswith("f_rest_"))
    if n_rest != 3 * (M - 1):  # gaussian_model.py:283 assert
        raise ValueError(f"PLY has {n_rest} f_rest_* properties, expected {3 * (M - 1)} for M={M}")
    col = [need(n) for n in ("x", "y", "z")]
    for m in range(M):  # arena features [M, 3]: file order is channel-major per block
        for c in range(3):
            col.append(need(f"f_dc_{c}") if m == 0 else need(f"f_rest_{c * (M - 1) + (m - 1)}"))
    col.append(need("opacity"))
    col += [need(f"scale_{j}") for j in range(3)]
    col += [need(f"rot_{j}") for j in range(4)]
    col += [need(f"segment_{j}") for j in range(C)]
    return col


def read_header(f):
    """Parse a PLY header from a binary file object; returns (format, elements,
    header_bytes) with elements = [(name, count, [(prop, numpy dtype str)])]."""
    first = f.readline()
    if first.strip() != b"ply":
        raise ValueError("not a PLY file")
    fmt, elements = None, []
    while True:
        line = f.readline()
        if not line:
            raise ValueError("PLY header has no end_header")
        tok = line.decode("ascii", "replace").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append((tok[1], int(tok[2]), []))
        elif tok[0] == "property":
            if tok[1] == "list":
                raise ValueError("PLY list properties are not supported in the vertex element")
            elements[-1][2].append((tok[2], _PLY_TYPES[tok[1]]))
        elif tok[0] == "end_header":
            return fmt, elements, f.tell()


def read_rows(path):
    """(names, float32 rows [n, F]) of the vertex element of a PLY file."""
    with open(path, "rb") as f:
        fmt, elements, hdr = read_header(f)
        if not elements or elements[0][0] != "vertex":
            raise ValueError("the first PLY element must be 'vertex'")
        _, n, props = elements[0]
        names = [p for p, _ in props]
        if fmt == "ascii":
            rows = np.loadtxt(f, dtype=np.float64, max_rows=n, ndmin=2).astype(np.float32)
            return names, np.ascontiguousarray(rows.reshape(n, len(props)))
    end = {"binary_little_endian": "<", "binary_big_endian": ">"}.get(fmt)
    if end is None:
        raise ValueError(f"unsupported PLY format {fmt!r}")
    if all(t == "f4" for _, t in props):
        rows = np.fromfile(path, dtype=end + "f4", count=n * len(props), offset=hdr).reshape(n, len(props))
        return names, np.ascontiguousarray(rows.astype("<f4", copy=False))
    rec = np.fromfile(path, dtype=np.dtype([(p, end + t) for p, t in props]), count=n, offset=hdr)
    rows = np.empty((n, len(props)), dtype=np.float32)
    for j, p in enumerate(names):
        rows[:, j] = rec[p]
    return names, rows


def write_rows(path, names, rows):
    """Binary little-endian PLY with one vertex element of float properties (what
    plyfile writes for the reference's save_ply)."""
    rows = np.ascontiguousarray(rows, dtype="<f4")
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {rows.shape[0]}"]
    head += [f"property float {n}" for n in names] + ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode("ascii"))
        rows.tofile(f)


def rows_to_arena(spec, param, rows_dev, names, dst=0):
    col = arena_columns(names, spec.M, spec.C)
    arr = (ctypes.c_int * len(col))(*col)
    n, F = rows_dev.shape
    _C._check(_lib.gsr_ply_rows_to_arena(n, F, rows_dev.data_ptr(), arr, spec.P, spec.M, spec.C, dst,
                                          param.data_ptr(), _C._stream(param.device)))


def arena_to_rows(spec, param, names):
    col = arena_columns(names, spec.M, spec.C)
    arr = (ctypes.c_int * len(col))(*col)
    rows = torch.empty((spec.P, len(names)), dtype=torch.float32, device=param.device)
    _C._check(_lib.gsr_arena_to_ply_rows(spec.P, spec.M, spec.C, param.data_ptr(), len(names), arr,
                                          rows.data_ptr() if spec.P else None, _C._stream(param.device)))
    return rows

