"""h5.py (the HDF5 subset under the cooler drop-in): the writer / in-place
append by round trips, and the reader on structures assembled here byte by
byte from the format specification (v2 object headers with link messages,
superblock v2).  The pin against the real libhdf5 -- files it wrote read
exactly, files h5.py writes read by it -- is tests/test_h5_libhdf5.py."""
import struct
import zlib

import numpy as np
import pytest

from hichap_master_amd import h5

UNDEF = h5.UNDEF


def _roundtrip_tree():
    rng = np.random.default_rng(0)
    return {
        "@attrs": {"format": "HDF5::Cooler", "format-version": 3, "nbins": 7, "ok": True, "no": False,
                   "scale": np.array([1.5, 2.5, 3.0]), "tol": 1e-5},
        "g": {
            "i8": rng.integers(-2**62, 2**62, size=50, dtype=np.int64),
            "i4": rng.integers(-2**31, 2**31 - 1, size=33, dtype=np.int32),
            "u2": rng.integers(0, 2**16, size=9).astype(np.uint16),
            "f8": rng.random(17),
            "f4": rng.random(5).astype(np.float32),
            "s": np.array([b"chr1", b"2", b"chrX_long"]),
            "m": rng.random((4, 6)),
            "scalar": np.float64(3.25),
            "with_attrs": {"@data": np.arange(4), "@attrs": {"unit": "bp", "n": 4}},
            "flags": np.array([True, False, True]),
        },
        "wide": {f"d{k:03d}": np.arange(k + 1) for k in range(40)},  # several symbol table nodes
        "empty_group": {},
    }


def test_write_read_roundtrip(tmp_path):
    p = str(tmp_path / "t.h5")
    tree = _roundtrip_tree()
    h5.write_file(p, tree)
    with h5.File(p) as f:
        assert sorted(f.root.keys()) == ["empty_group", "g", "wide"]
        a = f.root.attrs
        assert a["format"] == "HDF5::Cooler" and a["format-version"] == 3 and a["ok"] is True and a["no"] is False
        np.testing.assert_array_equal(a["scale"], [1.5, 2.5, 3.0])
        for k, v in tree["g"].items():
            d = f["g/" + k]
            if isinstance(v, dict):
                np.testing.assert_array_equal(d.read(), v["@data"])
                assert d.attrs == {"unit": "bp", "n": 4}
            else:
                np.testing.assert_array_equal(d.read(), v)
        np.testing.assert_array_equal(f["g/i8"].read(10, 20), tree["g"]["i8"][10:20])
        assert f["g/i4"].read(5, 5).size == 0
        assert sorted(f["wide"].keys()) == sorted(tree["wide"])
        for k, v in tree["wide"].items():
            np.testing.assert_array_equal(f["wide/" + k].read(), v)
        assert f["empty_group"].keys() == []
        with pytest.raises(KeyError):
            f["g/missing"]


def test_append_dataset_in_place(tmp_path):
    p = str(tmp_path / "a.h5")
    h5.write_file(p, {"bins": {"start": np.arange(6), "end": np.arange(6) + 1}, "other": {"x": np.zeros(3)}})
    w = np.linspace(0, 1, 6)
    h5.append_dataset(p, "bins", "weight", w, {"converged": True, "var": 1e-7, "scale": 12.5})
    with h5.File(p) as f:
        assert f["bins"].keys() == ["end", "start", "weight"]
        np.testing.assert_array_equal(f["bins/weight"].read(), w)
        assert f["bins/weight"].attrs == {"converged": True, "var": 1e-7, "scale": 12.5}
        np.testing.assert_array_equal(f["other/x"].read(), np.zeros(3))
    # --force: replace the column
    h5.append_dataset(p, "bins", "weight", -w, {"converged": False})
    # names sorting before / after the existing ones, and enough of them to
    # outgrow the local heap's spare block (the heap moves to the end)
    long = ["a" * 40, "zz" + "q" * 60, "m" * 70]
    for k, nm in enumerate(long):
        h5.append_dataset(p, "bins", nm, np.full(2, k))
    with h5.File(p) as f:
        assert f["bins"].keys() == sorted(["end", "start", "weight"] + long)
        np.testing.assert_array_equal(f["bins/weight"].read(), -w)
        assert f["bins/weight"].attrs == {"converged": False}
        for k, nm in enumerate(long):
            np.testing.assert_array_equal(f["bins/" + nm].read(), [k, k])
        np.testing.assert_array_equal(f["bins/start"].read(), np.arange(6))
    # past a symbol table node's 8 entries: the node splits (several times)
    extra = [f"n{k:02d}" for k in range(40)]
    for k, nm in enumerate(extra):
        h5.append_dataset(p, "bins", nm, np.full(1, k))
    with h5.File(p) as f:
        assert f["bins"].keys() == sorted(["end", "start", "weight"] + long + extra)
        for k, nm in enumerate(extra):
            np.testing.assert_array_equal(f["bins/" + nm].read(), [k])
        np.testing.assert_array_equal(f["bins/weight"].read(), -w)


# ---------------------------------------------------------------- hand-built
class _Img:
    def __init__(self):
        self.b = bytearray()

    def put(self, data, align=8):
        while len(self.b) % align:
            self.b.append(0)
        a = len(self.b)
        self.b += data
        return a

    def patch(self, at, data):
        self.b[at:at + len(data)] = data


def _v2_msgs(msgs):
    out = b""
    for t, d in msgs:
        out += struct.pack("<BHB", t, len(d), 0) + d
    return out


def _ohdr_v2(msgs):
    body = _v2_msgs(msgs)
    return b"OHDR" + bytes([2, 0x02]) + struct.pack("<I", len(body)) + body + b"\0\0\0\0"  # checksum unverified


def _dt_i4():
    return bytes([0x10, 0x08, 0, 0]) + struct.pack("<IHH", 4, 0, 32)


def test_reader_on_libhdf5_style_structures(tmp_path):
    """Superblock v2 + v2 object headers; a compact new-style root group
    (link messages); an int32 dataset chunked by 7 under a v1 B-tree with a
    shuffle + deflate pipeline (last chunk partial, one chunk with the
    deflate filter masked off); a variable-length UTF-8 string attribute in
    a global heap; an enum attribute; a scalar v2 dataspace."""
    rng = np.random.default_rng(3)
    data = rng.integers(-1000, 1000, size=23).astype("<i4")
    cs = 7
    img = _Img()
    img.put(b"\0" * 48)  # superblock v2 (patched below)
    # chunks
    chunks = []
    for k, s0 in enumerate(range(0, data.size, cs)):
        blk = np.zeros(cs, "<i4")
        part = data[s0:s0 + cs]
        blk[:part.size] = part
        shuf = np.frombuffer(blk.tobytes(), np.uint8).reshape(cs, 4).T.tobytes()
        mask = 2 if k == 1 else 0  # chunk 1 stored without the deflate step (filter index 1)
        raw = shuf if mask else zlib.compress(shuf, 6)
        chunks.append((s0, len(raw), mask, img.put(raw)))
    # v1 chunk B-tree, level 0
    bt = b"TREE" + bytes([1, 0]) + struct.pack("<HQQ", len(chunks), UNDEF, UNDEF)
    for s0, size, mask, addr in chunks:
        bt += struct.pack("<IIQQ", size, mask, s0, 0) + struct.pack("<Q", addr)
    bt += struct.pack("<IIQQ", 0, 0, data.size, 0)
    bt_at = img.put(bt)
    # global heap with one string object
    s = "HDF5::Cooler ünïcode".encode()
    obj = struct.pack("<HHIQ", 1, 1, 0, len(s)) + s + b"\0" * (h5._pad8(len(s)) - len(s))
    coll = b"GCOL" + bytes([1, 0, 0, 0]) + struct.pack("<Q", 16 + len(obj) + 16) + obj + b"\0" * 16
    gh_at = img.put(coll)
    # dataset object header (v2)
    dspace = bytes([2, 1, 1, 1]) + struct.pack("<QQ", data.size, UNDEF)
    layout = bytes([3, 2, 2]) + struct.pack("<Q", bt_at) + struct.pack("<II", cs, 4)
    filt = bytes([2, 2]) + struct.pack("<HHHI", 2, 0, 1, 4) + struct.pack("<HHHI", 1, 0, 1, 6)
    vlen_t = bytes([0x19, 0x01, 0, 0]) + struct.pack("<I", 16) + bytes([0x10, 0, 0, 0]) + struct.pack("<IHH", 1, 0, 8)
    scalar = bytes([2, 0, 0, 0])
    name = b"format\0"
    attr_s = bytes([3, 0]) + struct.pack("<HHH", len(name), len(vlen_t), len(scalar)) + bytes([1]) + name + vlen_t \
        + scalar + struct.pack("<IQI", len(s), gh_at, 1)
    enum_t = bytes([0x38, 2, 0, 0]) + struct.pack("<I", 1) + bytes([0x10, 0, 0, 0]) + struct.pack("<IHH", 1, 0, 8) \
        + b"FALSE\0TRUE\0" + bytes([0, 1])
    name2 = b"converged\0"
    attr_e = bytes([3, 0]) + struct.pack("<HHH", len(name2), len(enum_t), len(scalar)) + bytes([0]) + name2 + enum_t \
        + scalar + bytes([1])
    ds_at = img.put(_ohdr_v2([(0x01, dspace), (0x03, _dt_i4()), (0x08, layout), (0x0B, filt), (0x0C, attr_s),
                              (0x0C, attr_e)]))
    # root group: compact links (link info with no fractal heap + one link)
    linfo = bytes([0, 0]) + struct.pack("<QQ", UNDEF, UNDEF)
    link = bytes([1, 0x00, 5]) + b"count" + struct.pack("<Q", ds_at)
    root_at = img.put(_ohdr_v2([(0x02, linfo), (0x06, link)]))
    eof = len(img.b)
    img.patch(0, h5.SIG + bytes([2, 8, 8, 0]) + struct.pack("<QQQQ", 0, UNDEF, eof, root_at) + b"\0" * 4)
    p = tmp_path / "lib.h5"
    p.write_bytes(bytes(img.b))
    with h5.File(str(p)) as f:
        assert f.root.keys() == ["count"]
        d = f["count"]
        assert d.shape == (23,) and d.dtype == np.dtype("<i4")
        np.testing.assert_array_equal(d.read(), data)
        np.testing.assert_array_equal(d.read(5, 16), data[5:16])
        assert d.attrs == {"format": "HDF5::Cooler ünïcode", "converged": True}


def test_v1_header_continuation_and_contiguous(tmp_path):
    """v0 superblock, v1 object header whose messages continue in a second
    block (continuation message), contiguous float64 layout."""
    x = np.arange(10, dtype="<f8") / 3
    img = _Img()
    img.put(b"\0" * 96)
    data_at = img.put(x.tobytes())
    dspace = bytes([1, 1, 0, 0]) + b"\0" * 4 + struct.pack("<Q", 10)
    f8 = bytes([0x11, 0x20, 63, 0]) + struct.pack("<IHHBBBBI", 8, 0, 64, 52, 11, 0, 52, 1023)
    lay = bytes([3, 1]) + struct.pack("<QQ", data_at, x.nbytes)

    def m(t, d):
        d = d + b"\0" * (h5._pad8(len(d)) - len(d))
        return struct.pack("<HHB3x", t, len(d), 0) + d
    cont_body = m(0x08, lay)
    cont_at = img.put(cont_body)
    first = m(0x01, dspace) + m(0x03, f8) + m(0x10, struct.pack("<QQ", cont_at, len(cont_body)))
    ds_at = img.put(struct.pack("<BBHII", 1, 0, 4, 1, len(first)) + b"\0" * 4 + first)
    # root group: symbol table with one SNOD
    heap_data = b"\0" * 8 + b"x\0" + b"\0" * 6
    hd_at = img.put(heap_data)
    heap_at = img.put(b"HEAP" + bytes(4) + struct.pack("<QQQ", len(heap_data), UNDEF, hd_at))
    snod_at = img.put(b"SNOD" + bytes([1, 0]) + struct.pack("<H", 1) + struct.pack("<QQII16x", 8, ds_at, 0, 0))
    bt_at = img.put(b"TREE" + bytes([0, 0]) + struct.pack("<HQQ", 1, UNDEF, UNDEF) + struct.pack("<QQQ", 0, snod_at, 8))
    st = m(0x11, struct.pack("<QQ", bt_at, heap_at))
    root_at = img.put(struct.pack("<BBHII", 1, 0, 1, 1, len(st)) + b"\0" * 4 + st)
    eof = len(img.b)
    sb = h5.SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0) \
        + struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF) + struct.pack("<QQII16x", 0, root_at, 0, 0)
    img.patch(0, sb)
    p = tmp_path / "v1.h5"
    p.write_bytes(bytes(img.b))
    with h5.File(str(p)) as f:
        np.testing.assert_array_equal(f["x"].read(), x)
        np.testing.assert_array_equal(f["x"].read(3, 7), x[3:7])


def test_not_hdf5(tmp_path):
    p = tmp_path / "no.h5"
    p.write_bytes(b"plain text" * 100)
    with pytest.raises(h5.H5Error):
        h5.File(str(p))


def test_reader_2d_chunked_with_unallocated_chunk(tmp_path):
    """A 5 x 7 float64 dataset in 3 x 4 chunks (edge chunks partial), deflate
    only, one chunk never written (absent from the B-tree: reads as 0)."""
    x = np.arange(35, dtype="<f8").reshape(5, 7) / 7
    img = _Img()
    img.put(b"\0" * 48)
    entries = []
    for r0 in (0, 3):
        for c0 in (0, 4):
            if (r0, c0) == (3, 4):
                x[3:, 4:] = 0.0
                continue
            blk = np.zeros((3, 4), "<f8")
            part = x[r0:r0 + 3, c0:c0 + 4]
            blk[:part.shape[0], :part.shape[1]] = part
            raw = zlib.compress(blk.tobytes())
            entries.append((r0, c0, len(raw), img.put(raw)))
    bt = b"TREE" + bytes([1, 0]) + struct.pack("<HQQ", len(entries), UNDEF, UNDEF)
    for r0, c0, size, addr in entries:
        bt += struct.pack("<IIQQQ", size, 0, r0, c0, 0) + struct.pack("<Q", addr)
    bt += struct.pack("<IIQQQ", 0, 0, 5, 7, 0)
    bt_at = img.put(bt)
    dspace = bytes([2, 2, 0, 1]) + struct.pack("<QQ", 5, 7)
    f8 = bytes([0x11, 0x20, 63, 0]) + struct.pack("<IHHBBBBI", 8, 0, 64, 52, 11, 0, 52, 1023)
    layout = bytes([3, 2, 3]) + struct.pack("<Q", bt_at) + struct.pack("<III", 3, 4, 8)
    filt = bytes([2, 1]) + struct.pack("<HHHI", 1, 0, 1, 4)
    ds_at = img.put(_ohdr_v2([(0x01, dspace), (0x03, f8), (0x08, layout), (0x0B, filt)]))
    link = bytes([1, 0x00, 1]) + b"m" + struct.pack("<Q", ds_at)
    root_at = img.put(_ohdr_v2([(0x06, link)]))
    img.patch(0, h5.SIG + bytes([2, 8, 8, 0]) + struct.pack("<QQQQ", 0, UNDEF, len(img.b), root_at) + b"\0" * 4)
    p = tmp_path / "m.h5"
    p.write_bytes(bytes(img.b))
    with h5.File(str(p)) as f:
        np.testing.assert_array_equal(f["m"].read(), x)
