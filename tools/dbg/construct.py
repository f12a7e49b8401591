"""Debug: the traditional construction test with mismatch details."""
import json, os, sys, tempfile, pathlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from hichap_master_amd import _lib, matrixBuilding as mb, ice
from oracle import pairs_ref, cooler_ref, ice_ref
from tests.test_construction import _genome, _write_reps, _read_tables
_lib.load(); _lib.require_gpu()
g = dict(np.load("tests/golden/pairs_traditional.npz", allow_pickle=False))
p = json.loads(str(g["params"]))
gl = _genome(g)
tmp = pathlib.Path(tempfile.mkdtemp())
(tmp / "genome.txt").write_text("".join(gl))
reps = _write_reps(tmp, bytes(g["text"]))
coolers = mb.TraditionalMatrixConstruction(str(tmp), reps, str(tmp / "genome.txt"), p["wholeRes"], p["localRes"], p["chroms"])
for path in coolers:
    got = _read_tables(path)
    for res in got:
        cis = res in p["localRes"]
        t = got[res]
        b1, b2, cnt, w, off = t[1], t[2], t[3], t[5], t[6]
        wr, sr = ice_ref.balance(b1, b2, np.asarray(cnt).astype(np.int64), int(off[-1]), off, ignore_diags=1, cis_only=cis)
        wg, sg = ice.balance(b1, b2, np.asarray(cnt).astype(np.int64), int(off[-1]), off, ignore_diags=1, cis_only=cis)
        bad = np.flatnonzero(np.isnan(w) != np.isnan(wr))
        print(os.path.basename(path), res, "cis", cis, "n", off[-1], "nnz", b1.size, "nan got/ref/gpu-direct",
              np.isnan(w).sum(), np.isnan(wr).sum(), np.isnan(wg).sum(), "bad", bad[:10].tolist(),
              "iters", sr["iters"], sg["iters"], flush=True)
        if bad.size:
            print("   got", w[bad[:5]], "ref", wr[bad[:5]], "direct", wg[bad[:5]], "off", off.tolist()[:30])
