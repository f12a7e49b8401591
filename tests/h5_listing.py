"""Canonical listing of an HDF5 file as read by hichap_master_amd.h5, in the
format `make_h5_fixtures dump` prints from libhdf5 (tests/golden/
make_h5_fixtures.c): one line per group, dataset header, dataset values and
attribute; integers in decimal, floats as IEEE bit patterns in hex, strings
as the hex of their bytes.  Two listings are equal iff both readers see the
same tree, types, shapes, chunking, filters and values."""
import numpy as np

from hichap_master_amd import h5


def _tag(t):
    if t.vlen_str is not None:
        return "vstr"
    dt = t.dtype
    if t.enum is not None:
        base = f"{'u' if dt.kind == 'u' else 'i'}{dt.itemsize}"
        return f"enum({base})" + "{" + ",".join(f"{k}={int(v)}" for k, v in t.enum.items()) + "}"
    if dt.kind in "iu":
        return f"{dt.kind}{dt.itemsize}"
    if dt.kind == "f":
        return f"f{dt.itemsize}"
    if dt.kind == "S":
        return f"S{dt.itemsize}"
    return f"V{dt.itemsize}"


def _vals(t, arr):
    if t.vlen_str is not None:
        return ["x" + str(v).encode("utf-8").hex() for v in np.ravel(arr)]
    a = np.ascontiguousarray(np.asarray(arr, dtype=t.dtype)).ravel()
    if a.dtype.kind == "f":
        u = a.astype(a.dtype.newbyteorder("<")).view(f"<u{a.dtype.itemsize}")
        w = 2 * a.dtype.itemsize
        return [format(int(x), f"0{w}x") for x in u]
    if a.dtype.kind == "S":
        raw = a.tobytes()
        n = a.dtype.itemsize
        return ["x" + raw[k * n:(k + 1) * n].hex() for k in range(a.size)]
    return [str(int(x)) for x in a]


def _shape(shape):
    return "shape=(" + ",".join(str(int(d)) for d in (shape or ())) + ")"


def _attrs(node, path):
    out = []
    for name, typ, shape, val in node.attr_items():
        v = _vals(typ, val if shape else [val])
        out.append(f"A {path}@{name} {_tag(typ)} {_shape(shape)} =" + "".join(" " + x for x in v))
    return out


def listing(path):
    lines = []
    with h5.File(path) as f:
        def walk(node, p):
            if isinstance(node, h5.Dataset):
                lay = node.layout
                rank = len(node.shape or ())
                if lay[0] in ("chunked", "single", "indexed"):
                    dims = lay[2]
                    how = "chunked(" + ",".join(str(int(c)) for c in dims[:rank]) + ")"
                else:
                    how = lay[0]
                filt = "filters=[" + ",".join(str(fid) for fid, _ in node.filters) + "]"
                lines.append(f"D {p} {_tag(node.type)} {_shape(node.shape)} {how} {filt}")
                data = node.read()
                lines.append(f"V {p} =" + "".join(" " + x for x in _vals(node.type, data)))
            else:
                lines.append(f"G {p}")
                for k in node.keys():
                    walk(node[k], (p.rstrip("/") + "/" + k))
            lines.extend(_attrs(node, p))
        walk(f.root, "/")
    return sorted(lines)
