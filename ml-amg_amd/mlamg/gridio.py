"""Loader for the reference's `.grid` files (ns/model/data.py:208-243; ns/lib/helpers.py:18-20)
that executes nothing from the file.

A `.grid` is a bz2-compressed pickle of {'A': (data, indices, indptr), 'x': ndarray,
'extra': dict}. Instead of unpickling, this module walks the opcode stream (pickletools.genops,
a pure parser) with a tiny stack machine that only understands containers, scalars, strings,
bytes and the three globals numpy uses to serialise arrays (numpy.core.multiarray._reconstruct,
numpy.ndarray, numpy.dtype). Those globals are matched by name and never imported or called;
arrays are rebuilt from their raw byte payloads with numpy.frombuffer. Any other global or
opcode raises ValueError.
"""
from __future__ import annotations

import bz2
import pickletools

import numpy as np
import scipy.sparse as sp

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"): "reconstruct",
    ("numpy._core.multiarray", "_reconstruct"): "reconstruct",
    ("numpy", "ndarray"): "ndarray",
    ("numpy", "dtype"): "dtype",
}


class _Global:
    def __init__(self, kind):
        self.kind = kind


class _ArrayStub:
    def __init__(self):
        self.value = None


class _DtypeStub:
    def __init__(self, code):
        self.code = code
        self.order = None

    def dtype(self):
        dt = np.dtype(self.code)
        if self.order in ("<", ">"):
            dt = dt.newbyteorder(self.order)
        return dt


_MARK = object()


def _resolve(v):
    if isinstance(v, _ArrayStub):
        return v.value
    if isinstance(v, tuple):
        return tuple(_resolve(x) for x in v)
    if isinstance(v, list):
        return [_resolve(x) for x in v]
    if isinstance(v, dict):
        return {_resolve(k): _resolve(x) for k, x in v.items()}
    if isinstance(v, _DtypeStub):
        return v.dtype()
    return v


def parse_pickle_bytes(data: bytes):
    stack, memo = [], {}

    def pop_mark():
        items = []
        while True:
            v = stack.pop()
            if v is _MARK:
                break
            items.append(v)
        return items[::-1]

    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(_MARK)
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE",
                      "BININT", "BININT1", "BININT2", "LONG1", "BINFLOAT", "SHORT_BINSTRING",
                      "BINSTRING"):
            stack.append(arg)
        elif name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "TUPLE1":
            stack.append((stack.pop(),))
        elif name == "TUPLE2":
            b = stack.pop()
            a = stack.pop()
            stack.append((a, b))
        elif name == "TUPLE3":
            c = stack.pop()
            b = stack.pop()
            a = stack.pop()
            stack.append((a, b, c))
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name == "LIST":
            stack.append(list(pop_mark()))
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif name == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for k, v in zip(items[::2], items[1::2]):
                d[k] = v
        elif name == "STACK_GLOBAL":
            attr = stack.pop()
            mod = stack.pop()
            kind = _ALLOWED.get((mod, attr))
            if kind is None:
                raise ValueError(f"refusing pickle global {mod}.{attr}")
            stack.append(_Global(kind))
        elif name == "GLOBAL":
            mod, attr = arg.split(" ", 1)
            kind = _ALLOWED.get((mod, attr))
            if kind is None:
                raise ValueError(f"refusing pickle global {mod}.{attr}")
            stack.append(_Global(kind))
        elif name == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, _Global):
                raise ValueError("REDUCE on a non-global")
            if fn.kind == "reconstruct":
                stack.append(_ArrayStub())
            elif fn.kind == "dtype":
                stack.append(_DtypeStub(args[0]))
            else:
                raise ValueError(f"REDUCE on {fn.kind}")
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, _DtypeStub):
                obj.order = state[1]
            elif isinstance(obj, _ArrayStub):
                _ver, shape, dt, fortran, raw = state
                dt = dt.dtype() if isinstance(dt, _DtypeStub) else np.dtype(dt)
                if not isinstance(raw, (bytes, bytearray)):
                    raise ValueError("object arrays are not supported")
                arr = np.frombuffer(raw, dtype=dt).copy()
                arr = arr.reshape(shape, order="F" if fortran else "C")
                obj.value = arr
            else:
                raise ValueError("BUILD on an unsupported object")
        else:
            raise ValueError(f"unsupported pickle opcode {name}")
    if len(stack) != 1:
        raise ValueError("malformed pickle stream")
    return _resolve(stack[0])


def parse_grid_bytes(data: bytes):
    """Decoded (decompressed) .grid bytes -> dict with CSR arrays data/indices/indptr, x, extra."""
    obj = parse_pickle_bytes(data)
    A = obj["A"]
    if not isinstance(A, tuple):
        raise ValueError("only .grid files with A stored as (data, indices, indptr) are supported")
    data_, indices, indptr = A
    return {"data": data_, "indices": indices, "indptr": indptr, "x": obj.get("x"),
            "extra": obj.get("extra", {})}


def load_grid(path):
    """Grid.load (ns/model/data.py:223-235) without unpickling: returns (A csr, x, extra)."""
    if ".grid" not in path:
        path = path + ".grid"
    with bz2.open(path, "rb") as fh:
        g = parse_grid_bytes(fh.read())
    A = sp.csr_matrix((g["data"], g["indices"], g["indptr"]))
    extra = dict(g["extra"] or {})
    extra["filename"] = path
    return A, g["x"], extra
