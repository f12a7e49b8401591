"""ORACLE — test infrastructure only.

CPU restatements (NumPy) of the reference algorithms on the hot path:

* ``ice_ref``       — cooler's ICE balance as invoked by HiCHap
                      (``cooler balance --ignore-diags 1 [--cis-only]``,
                      matrixBuilding.py:708, :713, :1537, :1542, :1761, :1766).
                      cooler is a third-party package absent from
                      /root/reference and from this image: **parity unpinned**
                      for ICE (see ice_ref's header); pinned instead by
                      analytic known-answer tests.
* ``hichap_ref``    — HiCHap two-step / genome-wide correction
                      (matrixBuilding.py:742-1041).  Pinned against golden
                      vectors produced by the reference's own functions
                      (tests/golden/make_golden.py).
* ``structure_ref`` — compartment (StructureFind.py:201-460) and
                      directionality-index TAD scan (StructureFind.py:721-839).
                      Pinned against golden vectors as above.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / CPU baseline.  The
product package ``hichap_master_amd`` never imports it.
"""
