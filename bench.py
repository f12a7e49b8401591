#!/usr/bin/env python3
"""Benchmark: ICE iterations/s on the whole-genome 10 kb diploid matrix (C4).

Metric (BASELINE.json): "ICE iterations/sec + nnz·iters/sec on 10 kb
whole-genome matrix; 1/2/4/8 GPU".  Workload = configs[3]: hg19 chr1-22,X at
10 kb, maternal + paternal copies (607 282 bins), ~5e9 upper-triangle pixels
(20 % trans), generated directly in HBM (synthetic, SURVEY.md §8(d) model).

A step = one full ICE iteration (sweep over every pixel + variance + bias
update) with tol = 0 so no iteration is skipped.  N > 1: rows sharded across
ranks (one process per GPU), one all-gather of the marginal per iteration
over RCCL; total work fixed (strong scaling).  value = iterations/s of the
whole job; nnz_iters_per_s = pixels x iterations / s.

--config c5: the per-chromosome compartment path (configs[4]): hg19
autosomes at 25 kb as dense N x N float64 matrices generated in HBM, one
step = Distance_Decay + Get_PCA (O/E, Pearson on fp64 MFMA, top-3 PCA) +
Select_PC_new for all 22 autosomes; chromosomes dealt to ranks by LPT on N^3
(no collective); value = chromosomes/s of the whole job; roofline on k_syrk
(MFMA, fp64).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c4h|c3|c2|c1|c5|gw|dropin|e2e|pairs|loops]

--config c4h: the same metric on the haploid traditional 10 kb matrix (303 641 bins,
5e9 pixels), the one HiCHap's `cooler balance` runs on (matrixBuilding.py:1537).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_F64_MFMA_TFS = 78.6  # MI355X fp64 matrix spec (AMD datasheet; the guide has no fp64 row)
ALG_BYTES_PER_PIXEL = 12.0  # int32 bin1 + int32 bin2 + fp32 count


def measure_shard_sweep_ms(st, nloc, stream, n=5):
    """Average sweep time of this rank's shard (HIP-event registry), for the
    partition refinement; leaves the registry off and empty."""
    import torch
    from hichap_master_amd import _lib
    out = torch.zeros(max(int(nloc), 1), dtype=torch.float64, device="cuda")
    st.marg_local(2, out, stream)
    _lib.call("hh_ktime_reset")
    _lib.call("hh_ktime_enable", 1)
    for _ in range(n):
        st.marg_local(2, out, stream)
    torch.cuda.synchronize()
    _lib.call("hh_ktime_enable", 0)
    t, k = _lib.ktime("ice_sweep")
    _lib.call("hh_ktime_reset")
    return t / max(k, 1)


def config(name, nnz=None):
    from hichap_master_amd import synth
    if name == "c4":
        sizes = synth.genome_bins(10000, diploid=True)
        target, tf, label = nnz or 5e9, 0.2, "hg19-10kb-diploid-wholegenome"
    elif name == "c4h":
        # the haploid traditional T matrix HiCHap actually balances genome-wide
        # at 10 kb (matrixBuilding.py:1536-1538, :1760-1762): 3.04e5 bins
        # hg19 haploid at 10 kb has only 2.36e9 cis pairs in all, so 5e9
        # pixels need >= 53 % trans (0.6: A = 3.2e4, cis 85 % dense)
        sizes = synth.genome_bins(10000)
        target, tf, label = nnz or 5e9, 0.6, "hg19-10kb-haploid-wholegenome"
    elif name == "c3":
        sizes = synth.genome_bins(40000)
        # hg19 at 40 kb has only 1.42e8 cis pixels (sum n(n+1)/2, 2 % gaps), so
        # the ~8e8 nnz of BASELINE C3 needs ~85 % trans contacts
        target, tf, label = nnz or 8e8, 0.85, "hg19-40kb-wholegenome"
    elif name == "c2":
        sizes = [synth.chrom_bins([synth.HG19["1"]], 10000)[0]]
        target, tf, label = nnz or 5e7, 0.0, "hg19-chr1-10kb"
    elif name == "c1":
        sizes = [5000]
        target, tf, label = nnz or 2e6, 0.0, "single-chrom-40kb-5000-bins"
    elif name == "cis":
        # `cooler balance --cis-only` on the 10 kb file (matrixBuilding.py:713,
        # :1542, :1766): hg19 haploid, every chromosome its own ICE group, at
        # C2's per-chromosome density (chr1: 5e7 pixels) -> 6.1e8 cis pixels
        sizes = synth.genome_bins(10000)
        target, tf, label = nnz or 6.1e8, 0.0, "hg19-10kb-haploid-cisonly"
    else:
        raise SystemExit(f"unknown config {name}")
    A, td = synth.calibrate(sizes, target, tf)
    kw = dict(A=A, trans_density=td, comp_block=200, seed=20201015)
    if name == "cis":
        kw["cis_only"] = True
    return sizes, kw, label, target, tf


SWEEP_KERNELS = ("k_sweep_tiled", "k_sweep_flat", "k_sweep_band", "k_sweep_uband", "k_sweep_all")  # symmetric band: <8> once, <4> twice per sweep; upper band: <8>, <4> once each


# sources whose code decides a line's HBM traffic: a committed PMC summary
# counts for a run only when it was taken from these same sources on the same
# workload (a stale summary must not be reported as this run's)
_ICE_SOURCES = ("ice.hip", "ice_internal.hpp", "hh_common.hpp", "matrix.hip", "synth.hip", "build.hip")
PMC_SOURCES = {
    "c4": _ICE_SOURCES, "c4h": _ICE_SOURCES, "c3": _ICE_SOURCES, "c2": _ICE_SOURCES, "cis": _ICE_SOURCES,
    "gw": ("gw.hip", "pairs.hip", "hh_common.hpp", "ice_internal.hpp", "synth.hip"),
    "c5": ("comp.hip", "hh_common.hpp"),
    "twostep": ("dense.hip", "hh_common.hpp", "ice_internal.hpp"),
    "twostep_genome": ("dense.hip", "hh_common.hpp", "ice_internal.hpp"),
}


def src_sha(line):
    """sha256 over the sources of PMC_SOURCES[line] (hichap_master_amd/csrc)."""
    import hashlib
    h = hashlib.sha256()
    for f in PMC_SOURCES[line]:
        with open(os.path.join(ROOT, "hichap_master_amd", "csrc", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def pmc_pick(line, workload):
    """The committed PMC summary (profiles/*_<line>_pmc.json) whose _meta
    names this build's sources (src_sha) and this run's workload; None when
    none matches (the line then reports traffic null)."""
    import glob
    want = src_sha(line)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{line}_pmc.json")), reverse=True):
        data = json.load(open(f))
        meta = data.get("_meta") or {}
        wl = meta.get("workload") or {}
        if meta.get("src_sha") == want and all(wl.get(k) == v for k, v in workload.items()):
            return data, meta, os.path.relpath(f, ROOT)
    return None


def pmc_traffic(workload, kernels=SWEEP_KERNELS, line="c4"):
    """HBM bytes per ICE sweep (the sweep kernels, one launch each) from the
    committed rocprofv3 PMC summary of the `line` bench (c4, c4h, c3, c2,
    cis) taken at these sources on this workload (tools/pmc_summary.py), its
    metadata (commit, the layout's real bytes per sweep) and the file name;
    (None, None, None) without one."""
    got = pmc_pick(line, workload)
    if got is None:
        return None, None, None
    data, meta, src = got
    hits = [v for k, v in data.items() if k != "_meta" and any(name in k for name in kernels)]
    if not hits:
        return None, None, None
    # per sweep: a kernel launched k times per sweep (the 4-bit band's two
    # segments) has k times as many dispatches as the once-per-sweep kernels
    base = min(v.get("dispatches", 1) or 1 for v in hits)
    tot = sum(v["traffic_bytes"] * (v.get("dispatches", base) or base) / base for v in hits)
    return tot, meta, src


def gw_pmc_traffic(workload):
    """HBM bytes per genome-wide correction from the committed rocprofv3 PMC
    summary of the gw bench taken at these sources on this workload
    (profiles/*_gw_pmc.json, tools/pmc_summary.py): every kernel of the run
    except the synthetic-input generator, summed over its dispatches, divided
    by the number of corrections (the output-writing merge runs once per
    correction); (None, None) without one."""
    got = pmc_pick("gw", workload)
    if got is None:
        return None, None
    data, _, src = got
    runs = [v.get("dispatches", 0) for k, v in data.items() if k != "_meta" and "k_gw_merge" in k and "1>" in k]
    n_corr = max(runs) if runs else 0
    if not n_corr:
        return None, None
    tot = sum(v["traffic_bytes"] * v.get("dispatches", 0) for k, v in data.items()
              if k != "_meta" and "synth" not in k)
    return tot / n_corr, src


def twostep_pmc_traffic(line, workload):
    """HBM bytes per step of a TwoStep line (one hh_twostep_batch call: the
    chr1 device call or the whole 40 kb genome) from the committed PMC summary
    of that line at these sources on this workload (profiles/*_<line>_pmc.json):
    the batch kernels (k_rowstats_b, k_ts_*_b, k_sv_*_b; the bench's untimed
    host-array / pixel-table calls run other kernels) summed over their
    dispatches, divided by the dispatches of the output pass k_sv_out_b (one
    per batch call); (None, None) without one."""
    got = pmc_pick(line, workload)
    if got is None:
        return None, None
    data, _, src = got
    items = [(k, v) for k, v in data.items() if k != "_meta"]
    batch = [(k, v) for k, v in items if any(s in k for s in ("k_rowstats_b", "k_ts_gapdef_b", "k_ts_alpha_b",
                                                               "k_sv_"))]
    calls = sum(v.get("dispatches", 0) for k, v in batch if "k_sv_out_b" in k)
    if not calls:
        return None, None
    return sum(v["traffic_bytes"] * v.get("dispatches", 0) for k, v in batch) / calls, src


def c5_pmc_traffic(workload, kernels, primary, launches):
    """HBM bytes of one serial C5 pass in the kernels whose names contain any
    of `kernels` (rocprofv3 PMC summary of the C5 bench at these sources on
    this workload, profiles/*_c5_pmc.json): their bytes over the profiled run
    (per-dispatch average x dispatches, every template instance) divided by
    the passes that run held -- the `primary` kernel's dispatches over its
    `launches` per pass (HIP event registry); (None, None) without one."""
    got = pmc_pick("c5", workload)
    if got is None:
        return None, None
    data, _, src = got
    items = [(k, v) for k, v in data.items() if k != "_meta"]
    tot = sum(v["traffic_bytes"] * v.get("dispatches", 0) for k, v in items if any(s in k for s in kernels))
    nprim = sum(v.get("dispatches", 0) for k, v in items if primary in k)
    if not tot or not nprim or not launches:
        return None, None
    return tot / (nprim / float(launches)), src


def host_info():
    """The CPU every cpu_baseline ran on: model name and how many logical CPUs
    the machine has / this process may use (a GPU box shares its host)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"host_cpu_model": model, "host_nproc": os.cpu_count(), "host_cpus_usable": usable,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def with_host(d):
    d.update(host_info())
    return d


COOLER_NPROC = 8  # `cooler balance --nproc` default: HiCHap's call (matrixBuilding.py:708) passes none


def cpu_share():
    """Host CPUs this process may use for a CPU baseline: the box gives one
    GPU a share (OMP_NUM_THREADS, 16 on the GPU boxes), whatever nproc shows."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(usable, int(omp))) if omp and omp.isdigit() else usable


def cpu_baseline(sizes, kw, rc, nnz_total, label, budget_s=8.0):
    """Oracle (NumPy, cooler's bincount sweep) timed on the host on a bounded
    sample (the upper-triangle pixels of the first rows of the same matrix),
    at 1 process, at cooler's default process pool (8) and at this host's CPU
    share: each sweep's marginal split over forked workers as `cooler balance
    --nproc` does (oracle/ice_ref.sweep_rate_pool).  The reported value is
    the fastest of the three."""
    from hichap_master_amd import ice
    from oracle import ice_ref
    n = int(np.sum(sizes))
    per_row = max(nnz_total / n, 1.0)
    rows = int(min(n, max(64, 2.5e7 / per_row)))
    rows = min(n, (rows + 511) // 512 * 512)  # shards are whole 512-row blocks
    m = ice.ContactMatrix.synthetic(sizes, row_range=(0, rows), **kw)
    b1, b2, c = m.export_upper()
    m.close()

    def timed(fn):
        t0 = time.perf_counter()
        iters = 0
        while True:
            fn()
            iters += 1
            if time.perf_counter() - t0 > budget_s or iters >= 50:
                break
        return b1.size * iters / (time.perf_counter() - t0), iters

    share = cpu_share()
    runs = {1: timed(lambda: ice_ref.sweep_rate(b1, b2, c, n, 1))}
    for p in sorted({COOLER_NPROC, share} - {1}):
        runs[p] = timed(lambda p=p: ice_ref.sweep_rate_pool(b1, b2, c, n, 3, p))
        runs[p] = (runs[p][0] * 3, runs[p][1] * 3)  # 3 sweeps per pool (its start-up included)
    best = max(runs, key=lambda p: runs[p][0])
    pix_rate = runs[best][0]
    return {"value": pix_rate / nnz_total, "unit": f"ICE iterations/s (whole {label} matrix, extrapolated)",
            "cores": best, "kind": "port",
            "sample": f"oracle/ice_ref.sweep_rate(_pool) (numpy bincount, cooler restatement; the pool splits "
                      f"each sweep over forked workers as `cooler balance --nproc` does) on the {b1.size} upper "
                      f"pixels of rows [0,{rows}) of the same matrix; best of processes "
                      f"{sorted(runs)} = {best} at {pix_rate:.3g} pixel-iters/s",
            "pixel_iters_per_s": pix_rate,
            "by_processes": {str(p): {"pixel_iters_per_s": r, "iters_per_s_whole_matrix": r / nnz_total,
                                      "sweeps": it} for p, (r, it) in sorted(runs.items())},
            "cooler_default_nproc": COOLER_NPROC, "host_cpu_share": share}


def tad_scan_bench(m, st, stream, reps=5, res=10000, min_tad=200000, window=600000):
    """C2's TAD step after ICE: the gap + DI scan of the balanced chromosome
    (StructureFind.Data_preprocess :853-891 with HiCHap's defaults, minTAD
    200 kb and a 600 kb window) fed from the pixel table already in HBM
    (hh_tad_scan_pixels, on_device): band build + gap + DI, N x N never built."""
    import torch
    from hichap_master_amd._lib import call, ptr
    w, _ = st.finalize(stream)
    b1, b2, c = m.export_upper()
    n = int(m.info()["n_bins"])
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    d1, d2, dc, dw = dev(b1), dev(b2), dev(c.astype(np.float64)), dev(w)
    lb, wb = min_tad // res, window // res
    win = np.full(n, wb, np.int32)
    gap = np.empty(n, np.uint8)
    di = np.empty(n, np.float64)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call("hh_tad_scan_pixels", ptr(d1), ptr(d2), ptr(dc), b1.size, ptr(dw), n, 0, n, lb, ptr(win), 0,
             ptr(gap), ptr(di), 1, stream)
        ts.append(time.perf_counter() - t0)
    return {"ms": 1000.0 * float(np.median(ts[1:])), "pixels": int(b1.size), "bins": n, "band_halfwidth": wb,
            "gap_bins": int(gap.sum()), "nonzero_di": int(np.count_nonzero(di)),
            "what": "hh_tad_scan_pixels on device pixels + ICE weights: balanced band, Get_Gap, Get_DI (ttest)"}


C5_RES = 25000
C5_SCHED = os.environ.get("HH_C5_SCHED", "queue")  # "queue" (dynamic, largest first) or "static" (round-robin)
C5_STREAMS = int(os.environ.get("HH_C5_STREAMS", "12"))  # 12 host threads / streams: 95.8 vs 89.9 chr/s with 8 (profiles/r3b_c5b_s*.log)


def c5_sizes():
    from hichap_master_amd import synth
    return synth.chrom_bins([synth.HG19[str(c)] for c in range(1, 23)], C5_RES)


def c5_cpu_baseline(budget_chrom=20, seed=20201019):
    """Oracle compartment (NumPy corrcoef + exact SVD, numpy's BLAS threads)
    on the smallest autosome (chr21, hg19 25 kb) of the same synthetic model;
    extrapolated to the 22 autosomes by sum(N^3) / N_sample^3."""
    import torch
    from hichap_master_amd import ice
    from oracle import structure_ref
    sizes = c5_sizes()
    k = budget_chrom
    Nk = sizes[k]
    buf = torch.empty((Nk, Nk), dtype=torch.float64, device="cuda")
    ice.synth_dense(sizes, k, buf.data_ptr(), **c5_synth_kw())
    M = buf.cpu().numpy()
    t0 = time.perf_counter()
    structure_ref.compartment(M)
    dt = time.perf_counter() - t0
    cube = float(np.sum(np.asarray(sizes, dtype=float) ** 3))
    total = dt * cube / float(Nk) ** 3
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 1) for p in threadpool_info() if p.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    return {"value": len(sizes) / total, "unit": "chromosomes/s (22 hg19 autosomes at 25 kb, extrapolated)",
            "cores": threads, "kind": "port",
            "sample": f"oracle/structure_ref.compartment on chr21 (N={Nk}) of the same synthetic model: "
                      f"{dt:.2f}s; x sum(N^3)/N^3 = {total:.1f}s for the autosome set "
                      f"(numpy BLAS with {threads} threads)"}


def c5_synth_kw():
    return dict(A=120.0, trans_density=0.0, comp_block=80, ignore_diags=0, cis_only=True, gap_frac=0.02,
                seed=20201019)


def run_c5(args, world, rank, local):
    import torch
    from hichap_master_amd import _lib, dist, ice
    from hichap_master_amd.StructureFind import StructureFind
    sizes = c5_sizes()
    keys = list(range(len(sizes)))
    owner = dist.lpt_assign(np.asarray(sizes, dtype=float) ** 3, world)
    mine = [k for k in keys if owner[k] == rank]
    t0 = time.perf_counter()
    mats = {}
    for k in mine:
        mats[k] = torch.empty((sizes[k], sizes[k]), dtype=torch.float64, device="cuda")
        ice.synth_dense(sizes, k, mats[k].data_ptr(), **c5_synth_kw())
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    ng, prods, conv, phases = {}, {}, {}, {}
    # chromosomes run concurrently on C5_STREAMS HIP streams (one host thread
    # each; the C-ABI releases the GIL): the small chromosomes' PCA kernels are
    # latency-bound, so overlapping them keeps the GPU busy.
    from concurrent.futures import ThreadPoolExecutor
    streams = [torch.cuda.Stream(device=local) for _ in range(C5_STREAMS)]
    pool = ThreadPoolExecutor(max_workers=C5_STREAMS)

    def one(k, st):
        torch.cuda.set_device(local)  # the HIP current device is per host thread
        _lib.call("hh_set_device", local)
        with torch.cuda.stream(st):
            t_a = time.perf_counter()
            sf = StructureFind(Res=C5_RES, stream=st.cuda_stream)
            dec, G, NG = sf.Distance_Decay(M=mats[k], G_array=None)
            t_b = time.perf_counter()
            pcs, Cor, OE = sf.Get_PCA(distance_bin=dec, M=mats[k], NG_array=NG)
            t_c = time.perf_counter()
            sf.Select_PC_new(Cor, OE[NG], pcs)
            t_d = time.perf_counter()
            for key, v in (("decay", t_b - t_a), ("get_pca", t_c - t_b), ("select", t_d - t_c)):
                phases[key] = phases.get(key, 0.0) + v
            ng[k] = NG.size
            prods[k] = sf.pca_status["products"]
            conv[k] = sf.pca_status["converged"]

    def step(nstreams=C5_STREAMS):
        order = sorted(mine, key=lambda k: -sizes[k])
        if C5_SCHED == "static":  # largest first, dealt round-robin to the stream workers
            lanes = [order[i::nstreams] for i in range(nstreams)]
            futs = [pool.submit(lambda ks, st: [one(k, st) for k in ks], ks, st) for ks, st in zip(lanes, streams)]
        else:  # largest first from one queue: a worker takes the next chromosome when its stream is free
            import queue
            todo = queue.SimpleQueue()
            for k in order:
                todo.put(k)

            def worker(st):
                while True:
                    try:
                        k = todo.get_nowait()
                    except queue.Empty:
                        return
                    one(k, st)
            futs = [pool.submit(worker, st) for st in streams[:nstreams]]
        for f in futs:
            f.result()

    def barrier():
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t_start
    # per-kernel durations from one more pass with the streams serialised
    # (concurrent streams share the CUs, so their event spans overlap)
    phases.clear()
    t_ser = time.perf_counter()
    step(1)
    torch.cuda.synchronize()
    serial_ms = 1000.0 * (time.perf_counter() - t_ser)
    serial_phases = {k: round(1000.0 * v, 2) for k, v in phases.items()}
    _lib.call("hh_ktime_reset")
    _lib.call("hh_ktime_enable", 1)
    step(1)
    torch.cuda.synchronize()
    _lib.call("hh_ktime_enable", 0)
    syrk_ms, syrk_n = _lib.ktime("k_syrk")
    mul_ms, mul_n = _lib.ktime("k_cor_mul")
    orth_ms, orth_n = _lib.ktime("k_ortho")
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(tt.item())
    if rank == 0:
        flops = sum(float(sizes[k]) * ng[k] * (ng[k] + 1) for k in mine)  # one (serialised) pass
        syrk_tfs = flops / (syrk_ms / 1000.0) / 1e12 if syrk_ms > 0 else None
        # Cor . V products: HBM-bound stream of the padded ld x ld correlation,
        # its upper triangle of 64 x 64 tiles with k_cor_sym (hh_tune cor_sym, default on)
        ld = {k: (ng[k] + 127) // 128 * 128 for k in mine}
        cor_sym = "cor_sym=0" not in os.environ.get("HH_TUNE", "")
        if cor_sym:
            mul_bytes = sum(8.0 * 4096 * (ld[k] // 64) * (ld[k] // 64 + 1) / 2 * prods[k] for k in mine)
        else:
            mul_bytes = sum(8.0 * ld[k] * ld[k] * prods[k] for k in mine)
        mul_gbs = mul_bytes / (mul_ms / 1000.0) / 1e9 if mul_ms > 0 else None
        syrk_side = {"bound": "mfma", "kernel": "k_syrk", "achieved": syrk_tfs, "peak": PEAK_F64_MFMA_TFS,
                     "unit": "TFLOP/s", "frac": (syrk_tfs / PEAK_F64_MFMA_TFS) if syrk_tfs else None,
                     "total_ms": syrk_ms, "launches": syrk_n, "flops": flops}
        mul_side = {"bound": "hbm",
                    "kernel": "k_cor_sym (+ k_cor_sym_sum)" if cor_sym else "k_cor_mul_part (+ k_cor_mul_sum)",
                    "achieved": mul_gbs,
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": (mul_gbs / PEAK_HBM_GBS) if mul_gbs else None,
                    "total_ms": mul_ms, "launches": mul_n, "alg_bytes": mul_bytes,
                    "alg_bytes_note": ("8 B x the upper triangle of 64 x 64 tiles of the padded correlation per "
                                       "Cor.V product (k_cor_sym reads each off-diagonal tile once for both "
                                       "products; its partials, 2 x 128 B x (ld / 256 + 1) per row, are not counted)")
                    if cor_sym else "8 B x ld^2 (the padded correlation) per Cor.V product"}
        # the Krylov orthogonalisation (one k_ortho launch per product): per
        # cycle of P = 8 products block j reads the basis Q_0..Q_j twice (two
        # Gram-Schmidt passes) and W / its CholeskyQR iterates ~3 times, and
        # writes Q_{j+1}: ~(2 (j + 1) + 3) n x 16 x 8 B, 96 n x 128 B per cycle
        orth_bytes = sum(prods[k] / 8.0 * 96.0 * ng[k] * 128.0 for k in mine)
        orth_gbs = orth_bytes / (orth_ms / 1000.0) / 1e9 if orth_ms > 0 else None
        orth_side = {"bound": "latency (grid barriers)", "kernel": "k_ortho", "achieved": orth_gbs,
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": (orth_gbs / PEAK_HBM_GBS) if orth_gbs else None,
                     "total_ms": orth_ms, "launches": orth_n, "alg_bytes": orth_bytes,
                     "alg_bytes_note": "estimate: ~96 n x 128 B per Krylov cycle of 8 products (basis read twice, "
                                       "W and its CholeskyQR iterates, Q_{j+1} written); about 10 grid barriers "
                                       "per launch set its time"}
        # physical HBM bytes per serial pass from the committed PMC summary
        # (2 x FETCH_SIZE + WRITE_SIZE, the guide's gfx950 correction)
        wl = {"workload": "hg19-autosomes-25kb-compartment", "n_chroms": len(sizes),
              "bins_total": int(np.sum(sizes))}
        for side, names, prim, nl in ((orth_side, ("k_ortho",), "k_ortho", orth_n),
                                      (mul_side, ("k_cor_sym",) if cor_sym else ("k_cor_mul",),
                                       "k_cor_sym_pf" if cor_sym else "k_cor_mul_part", mul_n)):
            tr, src = c5_pmc_traffic(wl, names, prim, nl)
            side["traffic"] = tr
            side["traffic_source"] = src
            if tr and side["total_ms"]:
                side["traffic_GBps"] = tr / (side["total_ms"] / 1000.0) / 1e9
                side["traffic_frac"] = side["traffic_GBps"] / PEAK_HBM_GBS
        sides = sorted([syrk_side, mul_side, orth_side], key=lambda d: -(d["total_ms"] or 0.0))
        dom, other = sides[0], sides[1:]
        out = {
            "metric": "compartment PCA chromosomes/sec (C5: hg19 autosomes at 25 kb, dense per-chrom)",
            "value": len(sizes) * args.steps / elapsed, "unit": "chromosomes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic dense per-chrom matrices generated in HBM (SURVEY.md §8(d) model)",
            "config": {"workload": "hg19-autosomes-25kb-compartment", "n_chroms": len(sizes),
                       "bins_total": int(np.sum(sizes)), "largest_N": int(max(sizes)),
                       "parallelism": f"chromosomes LPT over {world} ranks" if world > 1 else "single GPU",
                       "generate_s": round(gen_s, 2),
                       "pca_products_per_chrom": {int(k) + 1: int(prods[k]) for k in sorted(mine)},
                       "pca_all_converged": bool(all(conv[k] for k in mine)),
                       "serial_step_ms": round(serial_ms, 2), "serial_phase_ms": serial_phases},
            "roofline": dict(dom, traffic=dom.get("traffic"),
                             kernel_timing="HIP events (hh_ktime) over one extra serialised pass after the timed steps; "
                                           "roofline = the kernel with the most time, other_kernels = the rest",
                             other_kernels=other),
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = with_host(c5_cpu_baseline())
        print(json.dumps(out), flush=True)


PAIRS_WHOLE = [10000]            # whole-genome matrix at the C4 resolution
PAIRS_LOCAL = [500000, 40000]    # HiCHap's default localRes (scripts/hichap:408)


def pairs_genome():
    from hichap_master_amd import synth
    return {c: synth.HG19[c] for c in synth.HG19_ORDER}


def synth_pairs_text(genome, n_lines, seed=20201016, fmt=0, line0=0):
    """Synthetic *_Valid.bed text generated in HBM (hh_synth_pairs_text)."""
    import ctypes as C
    import torch
    from hichap_master_amd._lib import call
    names = b"".join(b"chr" + c.encode() + b"\0" for c in genome)
    lens = np.array(list(genome.values()), dtype=np.int64)
    nb = C.c_int64(0)
    args = (len(genome), names, lens.ctypes.data_as(C.c_void_p), int(n_lines), 0.8, 1e8, fmt, seed, int(line0))
    call("hh_synth_pairs_text", *args, None, 0, C.byref(nb), None)
    buf = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    call("hh_synth_pairs_text", *args, C.c_void_p(buf.data_ptr()), nb.value, C.byref(nb), None)
    torch.cuda.synchronize()
    return buf


def pairs_cpu_baseline(genome, budget_s=10.0):
    """Oracle (oracle/pairs_ref.py: the reference's per-line loop restated,
    dict counts instead of dense += ) on a bounded sample of the same text."""
    from oracle import pairs_ref
    n = 4_000_000
    text = bytes(synth_pairs_text(genome, n, line0=0).cpu().numpy()).decode()
    lines = text.splitlines(keepends=True)
    t0 = time.perf_counter()
    done = 0
    step = 200_000
    while done < n and time.perf_counter() - t0 < budget_s:
        pairs_ref.traditional_counts(lines[done:done + step], genome, ["#", "X"], PAIRS_WHOLE, PAIRS_LOCAL)
        done += step
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"oracle/pairs_ref.traditional_counts (the reference's line loop, :566-596) on the first "
                      f"{done} lines of the same synthetic text: {dt:.1f}s"}


def run_pairs(args, world, rank, local):
    """Pair binning: synthetic hg19 *_Valid.bed text
    resident in HBM -> whole-genome 10 kb + intra-chromosome 500 kb / 40 kb
    pixel tables.  A step = parse + bin + sort + RLE of every pair; ranks
    bin disjoint line ranges of the same text (weak scaling, no collective:
    merging per-rank tables is the reference's replicate merge)."""
    import torch
    from hichap_master_amd import _lib, pairs
    genome = pairs_genome()
    n_lines = int(args.pairs)
    t0 = time.perf_counter()
    text = synth_pairs_text(genome, n_lines, line0=rank * n_lines)
    gen_s = time.perf_counter() - t0
    fmt = pairs.pairs_format(pairs.VALID_BED)
    stream = torch.cuda.current_stream().cuda_stream
    if os.environ.get("HH_PARSE_ABLATE"):  # timing ablations only (results wrong)
        _lib.call("hh_tune", b"parse_ablate", int(os.environ["HH_PARSE_ABLATE"]))
    info = {}

    def step():
        B = pairs.PairBinner(genome, ["#", "X"], stream=stream)
        ts = [B.add_target(r) for r in PAIRS_WHOLE] + [B.add_target(r, local=True) for r in PAIRS_LOCAL]
        B.feed_device(text.data_ptr(), text.numel(), fmt)
        B.finish()
        info["st"] = B.stats()
        info["nnz"] = []
        for t in ts:
            info["nnz"].append((t.res, t.local) + B.sizes(t))
        B.close()

    def barrier():
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t_start
    _lib.call("hh_ktime_reset")
    _lib.call("hh_ktime_enable", 1)
    step()
    torch.cuda.synchronize()
    _lib.call("hh_ktime_enable", 0)
    kt = {k: _lib.ktime(k) for k in ("k_parse_tile", "k_rs_hist", "k_rs_scatter")}
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(tt.item())
    if rank == 0:
        text_bytes = int(text.numel())
        keys_total = sum(x[3] for x in info["nnz"])
        # dominant-kernel roofline: the parse reads every text byte once and
        # writes one 8 B key per pair and target; the radix scatter reads and
        # writes 8 B per key per pass (+ the hist pass reads 8 B)
        parse_ms, _ = kt["k_parse_tile"]
        scat_ms, scat_n = kt["k_rs_scatter"]
        hist_ms, _ = kt["k_rs_hist"]
        parse_bytes = text_bytes + 8.0 * keys_total
        passes_bytes = 24.0 * sum(x[3] * ((2 * (int(np.ceil(np.log2(max(2, _nbins(genome, x[0]))))) ) + 7) // 8)
                                  for x in info["nnz"])
        dom = "k_parse_tile" if parse_ms >= scat_ms + hist_ms else "k_rs_hist+k_rs_scatter"
        if dom == "k_parse_tile":
            achieved = parse_bytes / (parse_ms / 1000.0) / 1e9
        else:
            achieved = passes_bytes / ((scat_ms + hist_ms) / 1000.0) / 1e9
        out = {
            "metric": "pair binning pairs/sec (Valid.bed text in HBM -> cooler pixel tables)",
            "value": world * n_lines * args.steps / elapsed, "unit": "pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic hg19 *_Valid.bed text generated in HBM (15 columns, 80% cis, log-uniform distance)",
            "config": {"workload": "hg19-validbed-pairs", "pairs_per_rank": n_lines, "text_bytes_per_rank": text_bytes,
                       "whole_res": PAIRS_WHOLE, "local_res": PAIRS_LOCAL,
                       "targets": [{"res": r, "local": bool(l), "pixels": nz, "pairs": npair}
                                   for r, l, nz, npair in info["nnz"]],
                       "stats": info["st"], "generate_s": round(gen_s, 2)},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                         "kernel_ms": {k: v[0] for k, v in kt.items()},
                         "parse_alg_bytes": parse_bytes, "sort_alg_bytes": passes_bytes,
                         "kernel_timing": "HIP events (hh_ktime) over one extra step after the timed steps"},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = with_host(pairs_cpu_baseline(genome))
        print(json.dumps(out), flush=True)


def _nbins(genome, res):
    return sum(l // res + 1 for l in genome.values())


LOOPS_RES = 10000


def loops_band(N, res, seed=20201018, depth=60.0):
    """Synthetic raw band (N x num) of one chromosome: power-law decay,
    log-normal visibility, planted loop pixels, 1 % empty bins; weights =
    1 / sqrt(row sum) (NaN for empty bins).  Band-only: no N x N matrix."""
    from hichap_master_amd import loops
    p = loops.peaks_parameter(res)
    num = p["maxapart"] // res + p["maxww"] + 1
    rng = np.random.default_rng(seed)
    vis = rng.lognormal(0, 0.2, N)
    d = np.arange(num)[None, :]
    r = np.arange(N)[:, None]
    inside = (r + d) < N
    lam = depth * (d + 1.0) ** -1.0 * vis[:, None] * vis[np.minimum(r + d, N - 1)]
    for _ in range(N // 40):
        a = int(rng.integers(5, N - num))
        b = int(rng.integers(p["ww"] + 2, num - 4))
        lam[a - 1:a + 2, b - 1:b + 2] *= 4.0
    Hb = np.where(inside, rng.poisson(lam), 0)
    gaps = rng.choice(N, size=N // 100, replace=False)
    Hb[gaps, :] = 0
    for g in gaps:  # column g of the band matrix
        rows = np.arange(max(0, g - num + 1), g + 1)
        Hb[rows, g - rows] = 0
    rs = Hb.sum(1).astype(float)
    w = np.where(rs > 0, 1.0 / np.sqrt(np.maximum(rs, 1.0)), np.nan)
    return Hb, w, num


def loops_dense_from_band(Hb):
    N, num = Hb.shape
    H = np.zeros((N, N), dtype=np.int64)
    r = np.repeat(np.arange(N), num)
    c = r + np.tile(np.arange(num), N)
    ok = c < N
    H[r[ok], c[ok]] = Hb.ravel()[ok]
    H[c[ok], r[ok]] = Hb.ravel()[ok]
    return H


def run_loops(args, world, rank, local):
    """HICCUPS on hg19 chr1 at 10 kb: one step = the
    window-widening loop (donut / lower-left sums of every candidate pixel,
    one launch per width, the reference's stop rule) over bands resident in
    HBM.  Ranks run independent chromosomes (weak scaling, no collective)."""
    import torch
    from hichap_master_amd import _lib, loops, synth
    N = synth.chrom_bins([synth.HG19["1"]], LOOPS_RES)[0]
    t0 = time.perf_counter()
    Hb, w, num = loops_band(N, LOOPS_RES, seed=20201018 + rank)
    H = loops_dense_from_band(Hb)
    t_wall = time.perf_counter()
    D, L, widths = loops.pcaller(H, w, LOOPS_RES, return_widths=True)   # whole chromosome, host glue included
    wall_s = time.perf_counter() - t_wall
    B = loops.bands(H, w, LOOPS_RES)
    del H
    xi, yi = loops.candidates(B)
    nb = loops.Neighbourhood(B)
    nb.set_pixels(xi, yi)
    gen_s = time.perf_counter() - t0

    def step():
        nb.reset()
        nb.widen()

    def barrier():
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t_start
    _lib.call("hh_ktime_reset")
    _lib.call("hh_ktime_enable", 1)
    step()
    torch.cuda.synchronize()
    _lib.call("hh_ktime_enable", 0)
    k_ms, k_n = _lib.ktime("k_hiccups_width")
    nb.close()
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(tt.item())
    if rank == 0:
        n = int(xi.size)
        prefix_bytes = 3.0 * N * (num + 1) * 8.0  # the three prefix arrays, read once per launch at best
        k_avg = k_ms / max(k_n, 1) / 1000.0
        achieved = prefix_bytes / k_avg / 1e9 if k_avg > 0 else None
        out = {
            "metric": "HICCUPS candidate pixels/sec (window-widening neighbourhood sums, hg19 chr1 10 kb)",
            "value": world * n * args.steps / elapsed, "unit": "pixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic chr1 band (power-law decay, planted loops) generated on the host",
            "config": {"workload": "hg19-chr1-10kb-hiccups", "bins": int(N), "band_diagonals": int(num),
                       "candidates": n, "widths": widths, "calls": len(D),
                       "pcaller_wall_s_incl_host_glue": round(wall_s, 3), "setup_s": round(gen_s, 2),
                       "parallelism": f"independent chromosomes x{world}" if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "kernel": "k_hiccups_width", "achieved": achieved, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS if achieved else None, "traffic": None,
                         "launches_per_step": k_n, "kernel_ms_avg": k_avg * 1000.0,
                         "alg_bytes_per_launch": prefix_bytes,
                         "note": "gather-bound (L2/MALL): ~150 prefix lookups per pixel per width"},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = with_host(loops_cpu_baseline())
        print(json.dumps(out), flush=True)


def loops_cpu_baseline(budget_s=12.0):
    """Oracle (oracle/loops_ref.py: the reference's window loop restated with
    dense-band gathers per offset) on an 8000-bin piece of the same model."""
    from hichap_master_amd import loops
    from oracle import loops_ref
    Hb, w, num = loops_band(8000, LOOPS_RES, seed=7)
    H = loops_dense_from_band(Hb)
    P = loops_ref.prepare(H, w, LOOPS_RES)
    xi, yi = loops_ref.candidates(P)
    t0 = time.perf_counter()
    loops_ref.neighbourhood(P, xi, yi)
    dt = time.perf_counter() - t0
    return {"value": xi.size / dt, "unit": "pixels/s", "cores": 1, "kind": "port",
            "sample": f"oracle/loops_ref.neighbourhood on an 8000-bin chromosome of the same model "
                      f"({xi.size} candidates) in {dt:.1f}s (NumPy; the reference's own scipy.sparse "
                      f"shifted-diagonal sums are slower still)"}


def run_dropin(args, world, rank, local):
    """The drop-in path as a HiCHap user reaches it: cooler's
    pixel table on the HOST (int32 bin1 / bin2 / count, sorted, as
    ``cooler.Cooler(uri).pixels()`` holds it) -> upload -> device layout build
    -> filters -> ICE, each phase timed.  Workload: C3 (hg19 40 kb whole
    genome, 8e8 pixels; the synthetic matrix's pixel table is exported once to
    the host first, untimed).  A step = the whole chain; ICE runs cooler's
    defaults (tol 1e-5, max 200 iterations) unless --fixed-iters."""
    import torch
    from hichap_master_amd import ice
    sizes, kw, label, target, tf = config("c3", args.nnz)
    n = int(np.sum(sizes))
    m = ice.ContactMatrix.synthetic(sizes, **kw)
    b1, b2, c = m.export_upper()
    m.close()
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    hb1, hb2, hc = (np.ascontiguousarray(x, dtype=np.int32) for x in (b1, b2, c))
    del b1, b2, c
    nnz = hb1.size
    opts = ice.IceOptions(max_iters=args.iters, tol=0.0 if args.fixed_iters else 1e-5)
    stream = torch.cuda.current_stream().cuda_stream
    phases = {}

    def step():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = [torch.from_numpy(x).to("cuda", non_blocking=False) for x in (hb1, hb2, hc)]
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        mm = ice.ContactMatrix.from_device_pixels(d[0], d[1], d[2], n, off, stream=stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        del d
        w, st = ice.balance_matrix(mm, opts, stream)
        t3 = time.perf_counter()
        mm.close()
        for k, v in (("upload_s", t1 - t0), ("build_s", t2 - t1), ("filters_and_ice_s", t3 - t2),
                     ("ice_sweeps_s", st["sweep_seconds"])):
            phases.setdefault(k, []).append(v)
        phases.setdefault("iters", []).append(st["iters"])
        return w

    for _ in range(args.warmup):
        step()
    phases.clear()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    elapsed = time.perf_counter() - t_start
    if rank == 0:
        med = {k: float(np.median(v)) for k, v in phases.items()}
        up_bytes = 12.0 * nnz
        out = {
            "metric": "cooler-balance drop-in: host pixel table -> weights (C3, hg19 40 kb whole genome)",
            "value": args.steps / elapsed, "unit": "balanced matrices/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "replicas", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic C3 pixel table (SURVEY.md §8(d) model) exported to host int32 arrays",
            "config": {"workload": label + "-host-pixel-table", "n_bins": n, "pixels": int(nnz),
                       "ice": "tol 0 (fixed iterations)" if args.fixed_iters else "cooler defaults (tol 1e-5)",
                       "max_iters": args.iters},
            "phases_median": med,
            "upload_GBps": up_bytes / med["upload_s"] / 1e9,
            "build_pixels_per_s": nnz / med["build_s"],
            "note": "upload = pageable host int32 -> HBM (PCIe); build = hh_matrix_from_pixels_device "
                    "(validate, filters, lower-half radix sort, tiles/bands); filters_and_ice = hh_ice_balance",
        }
        print(json.dumps(out), flush=True)


def run_e2e(args, world, rank, local):
    """pairs -> weights with nothing on the host: synthetic *_Valid.bed text in
    HBM -> PairBinner (whole-genome target at --res) -> ContactMatrix (device
    build from the binner's table) -> ICE (cooler defaults).  The chain of
    TraditionalMatrixConstruction + `cooler balance` (matrixBuilding.py:617-714)
    without the cooler file.  A step = the whole chain."""
    import torch
    from hichap_master_amd import ice, pairs
    genome = pairs_genome()
    n_lines = int(args.pairs)
    text = synth_pairs_text(genome, n_lines, line0=rank * n_lines)
    fmt = pairs.pairs_format(pairs.VALID_BED)
    stream = torch.cuda.current_stream().cuda_stream
    opts = ice.IceOptions(max_iters=args.iters, tol=1e-5)
    phases, info = {}, {}

    def step():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        B = pairs.PairBinner(genome, ["#", "X"], stream=stream)
        t = B.add_target(args.res)
        B.feed_device(text.data_ptr(), text.numel(), fmt)
        B.finish()
        t1 = time.perf_counter()
        mm = B.contact_matrix(t)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        w, st = ice.balance_matrix(mm, opts, stream)
        t3 = time.perf_counter()
        info.update(pixels=B.sizes(t)[0], bins=t.n_bins, iters=st["iters"], converged=st["converged"],
                    payload_bytes=mm.info()["payload_bytes"])
        mm.close()
        B.close()
        for k, v in (("bin_s", t1 - t0), ("build_s", t2 - t1), ("filters_and_ice_s", t3 - t2),
                     ("ice_sweeps_s", st["sweep_seconds"])):
            phases.setdefault(k, []).append(v)

    for _ in range(args.warmup):
        step()
    phases.clear()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    elapsed = time.perf_counter() - t_start
    if rank == 0:
        out = {
            "metric": "pairs -> ICE weights end to end (Valid.bed text in HBM, whole genome)",
            "value": n_lines * args.steps / elapsed, "unit": "pairs/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "replicas", "vs_baseline": None, "dtype": "int64/f64",
            "data": "synthetic hg19 *_Valid.bed text generated in HBM",
            "config": {"workload": f"hg19-validbed-{args.res // 1000}kb-wholegenome-balance", "pairs": n_lines,
                       "res": args.res, **info},
            "phases_median": {k: float(np.median(v)) for k, v in phases.items()},
        }
        print(json.dumps(out), flush=True)


def run_gw(args, world, rank, local):
    """Sparse GenomeWideMatrixCorrection (matrixBuilding.py:857-901) at the C4
    resolution: hg19 10 kb, T = the haploid whole-genome table (n = 303 641
    bins), H = the imputed diploid matrix as ordered asymmetric cells (2n =
    607 282 bins), both generated in HBM; the reference's dense form would
    need 2.9 TB per matrix.  A step = the whole correction: validate + column
    sort + integer statistics, the host alpha glue, S / symmetrise / VC^(2/3)
    / rescale into the upper-triangle table."""
    import torch
    from hichap_master_amd import _lib, ice, synth
    from hichap_master_amd.matrixBuilding import GenomeWideMatrixCorrectionSparse
    names = synth.HG19_ORDER
    nb = synth.genome_bins(10000)
    n = int(np.sum(nb))
    t_target, h_target = args.gw_t, args.gw_h
    At, tdt = synth.calibrate(nb, t_target, 0.2)
    Ah, tdh = synth.calibrate(nb + nb, h_target / 2.0, 0.2)
    t0 = time.perf_counter()
    T = ice.SynthPixels(nb, ordered=False, A=At, trans_density=tdt, comp_block=200, ignore_diags=0, seed=20201021)
    H = ice.SynthPixels(nb + nb, ordered=True, A=Ah, trans_density=tdh, comp_block=200, ignore_diags=0,
                        seed=20201022)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    off = np.concatenate([[0], np.cumsum(nb)])
    bins = {c: (int(off[k]), int(off[k + 1]) - 1) for k, c in enumerate(names)}
    hap = {}
    for k, c in enumerate(names):
        hap["M" + c] = bins[c]
        hap["P" + c] = (n + bins[c][0], n + bins[c][1])
    info = {}

    def step():
        out = GenomeWideMatrixCorrectionSparse(bins, hap, (T.bin1, T.bin2, T.count), (H.bin1, H.bin2, H.count),
                                               device_result=True)
        info["out_nnz"] = int(out[0].numel())
        del out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if rank == 0:
        in_bytes = 12.0 * (T.nnz + H.nnz)
        out_bytes = 16.0 * info["out_nnz"]  # int32 bin1 + int32 bin2 + fp64 value
        step_s = elapsed / args.steps
        alg = in_bytes + out_bytes
        # physical HBM bytes per correction (2 x FETCH_SIZE + WRITE_SIZE over
        # every kernel, MI355X_MICROARCH.md's gfx950 correction), when a PMC
        # summary of this line is committed
        gw_traffic, gw_traffic_src = gw_pmc_traffic({"T_pixels": T.nnz, "H_cells": H.nnz})
        out = {
            "metric": "sparse GenomeWideMatrixCorrection, hg19 10 kb diploid (T table + imputed H cells -> corrected table)",
            "value": args.steps / elapsed, "unit": "corrections/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "replicas", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic T (upper table) and H (ordered asymmetric cells) generated in HBM",
            "config": {"workload": "hg19-10kb-diploid-genomewide-correction", "n_bins_T": n, "n_bins_H": 2 * n,
                       "T_pixels": T.nnz, "H_cells": H.nnz, "out_pixels": info["out_nnz"],
                       "generate_s": round(gen_s, 2)},
            "input_GBps": in_bytes / step_s / 1e9,
            "cells_per_s": H.nnz * args.steps / elapsed,
            "roofline": {"bound": "hbm", "kernel": "the whole correction (hh_gw_create + hh_gw_correct: ~25 kernels, "
                                                   "per-kernel times in profiles/*gw_kernel_stats.csv)",
                         "achieved": alg / step_s / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": alg / step_s / 1e9 / PEAK_HBM_GBS, "traffic": gw_traffic,
                         "traffic_source": gw_traffic_src,
                         "traffic_GBps": gw_traffic / step_s / 1e9 if gw_traffic else None,
                         "traffic_note": "2 x FETCH_SIZE + WRITE_SIZE summed over the correction's kernels (the "
                                         "gfx950 doubling assumes wide streaming reads, so the gathers' share "
                                         "- alpha / s lookups in the marginals and merges - is an upper bound)",
                         "alg_bytes_per_launch": alg,
                         "alg_bytes_note": "12 B per T pixel and H cell read (int32 ids, int32 count) + 16 B per "
                                           "corrected upper cell written (int32 bin1, bin2, fp64 value)"},
            "note": "dense reference form: 607282^2 x 8 B = 2.9 TB per matrix (infeasible)",
        }
        if not args.no_cpu:
            out["cpu_baseline"] = with_host(gw_cpu_baseline(bins, hap, H.nnz))
            out["vs_cpu_baseline"] = out["value"] / out["cpu_baseline"]["value"]
        print(json.dumps(out), flush=True)
    T.close()
    H.close()


def gw_cpu_baseline(bins, hap, h_full, depth=2e8, seed=20201023):
    """The pixel-table oracle (oracle/hichap_ref.genome_wide_correction_sparse,
    NumPy, 1 core) on the same 10 kb diploid layout at reduced depth (~2e8 T
    pixels + ~2e8 H cells, generated on the GPU and copied to the host; at
    much lower depth whole chromosomes fall under Gap_definedLowRes's 0.1
    coverage and the reference's alpha step raises), as corrections/s
    extrapolated by H cells."""
    import ctypes as C
    import torch
    from hichap_master_amd import ice, synth
    from hichap_master_amd._lib import call
    from oracle import hichap_ref
    nb = synth.genome_bins(10000)
    At, tdt = synth.calibrate(nb, depth, 0.2)
    Ah, tdh = synth.calibrate(nb + nb, depth / 2.0, 0.2)
    T = ice.SynthPixels(nb, ordered=False, A=At, trans_density=tdt, comp_block=200, ignore_diags=0, seed=seed)
    H = ice.SynthPixels(nb + nb, ordered=True, A=Ah, trans_density=tdh, comp_block=200, ignore_diags=0,
                        seed=seed + 1)

    def host(a):
        t = torch.empty(a.numel(), dtype=torch.int32, device="cuda")
        if a.numel():
            call("hh_device_copy", C.c_void_p(t.data_ptr()), C.c_void_p(a.data_ptr()), 4 * a.numel(), None)
        call("hh_synchronize", None)
        return t.cpu().numpy()

    tp = tuple(host(x) for x in (T.bin1, T.bin2, T.count))
    hc = tuple(host(x) for x in (H.bin1, H.bin2, H.count))
    hn = H.nnz
    T.close()
    H.close()
    t0 = time.perf_counter()
    hichap_ref.genome_wide_correction_sparse(bins, hap, tp, hc)
    dt = time.perf_counter() - t0
    return {"value": (hn / dt) / h_full, "unit": "corrections/s (full-depth matrix, extrapolated by H cells)",
            "cores": 1, "kind": "port",
            "sample": f"oracle/hichap_ref.genome_wide_correction_sparse (NumPy) on the 10 kb diploid layout at "
                      f"{tp[0].size} T pixels + {hn} H cells: {dt:.1f} s = {hn / dt:.3g} H cells/s",
            "cells_per_s": hn / dt}


def run_twostep(args, world, rank, local):
    """TwoStepCorrection (matrixBuilding.py:984-1023) at HiCHap's default
    localRes: hg19 chr1 at 40 kb (N = 6 232), synthetic T / imputed M, P.
    A step = the whole correction on device-resident int64 matrices (gaps,
    alpha, gap-aware symmetrisation, VC^(2/3), mean rescale; no host round
    trip).  Also timed: the host-array call (3 uploads + 2 downloads of
    N^2 x 8 B) and the cell-fed call (pixel tables in, upper tables out)."""
    import torch
    from hichap_master_amd import matrixBuilding as mb, synth
    N = 249250621 // 40000 + 1
    rng = np.random.default_rng(20201024)
    TM = synth.dense_chrom(N, rng, A=60.0)
    MM, PM = synth.haplotype_pair(TM, rng, drop_rows=120)
    dev = [torch.from_numpy(X).cuda() for X in (TM, MM, PM)]
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        mb.TwoStepCorrection(*dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = mb.TwoStepCorrection(*dev)
        del out
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step = elapsed / args.steps
    # the host-array form and the cell-fed form (a few calls each)
    def wall(fn, k=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / k
    i, j = np.nonzero(np.triu(TM))
    tp = (i, j, TM[i, j])
    cells = []
    for X in (MM, PM):
        r, c = np.nonzero(X)
        cells.append((r, c, X[r, c]))
    # (--main-only, the PMC passes: no other calls, so every batch dispatch
    # in the profile is a step's)
    host_s = None if args.main_only else wall(lambda: mb.TwoStepCorrection(TM, MM, PM))
    cells_s = None if args.main_only else wall(lambda: mb.TwoStepCorrectionPixels(N, tp, cells[0], cells[1]))
    alg = 3 * 8.0 * N * N + 2 * 8.0 * N * N  # 3 int64 reads + 2 fp64 writes
    if rank == 0:
        out = {"metric": "TwoStepCorrection, hg19 chr1 at 40 kb (N = 6232), device-resident",
               "value": 1.0 / step, "unit": "chromosomes/s", "n_gpus": 1, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1000.0 * step, "higher_is_better": True,
               "scaling": "replicas", "vs_baseline": None, "dtype": "int64 in, f64 out",
               "data": "synthetic (synth.dense_chrom + haplotype_pair)",
               "config": {"workload": "twostep-chr1-40kb", "N": N, "nnz_T_upper": int(i.size),
                          "cells_MM": int(cells[0][0].size), "cells_PM": int(cells[1][0].size)},
               "roofline": {"bound": "hbm", "kernel": "hh_twostep (k_rowstats x3, k_symvc passes x2 matrices)",
                            "achieved": alg / step / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": alg / step / 1e9 / PEAK_HBM_GBS, "traffic": None,
                            "alg_bytes_per_launch": alg},
               "host_arrays_ms": None if args.main_only else 1000.0 * host_s,
               "cells_in_upper_out_ms": None if args.main_only else 1000.0 * cells_s,
               "note": "host_arrays_ms: numpy N x N in / out (PCIe: 1.55 GB per call); cells_in_upper_out_ms: "
                       "pixel tables in, corrected upper tables out (TwoStepCorrectionPixels)"}
        tr, tr_src = twostep_pmc_traffic("twostep", {"workload": "twostep-chr1-40kb", "N": N})
        if tr:
            out["roofline"].update(traffic=tr, traffic_source=tr_src, traffic_GBps=tr / step / 1e9,
                                   traffic_frac=tr / step / 1e9 / PEAK_HBM_GBS,
                                   traffic_note="2 x FETCH_SIZE + WRITE_SIZE of the batch kernels per call")
        if not args.no_cpu:
            from oracle import hichap_ref
            t = time.perf_counter()
            hichap_ref.two_step_correction(TM, MM, PM)
            dt = time.perf_counter() - t
            out["cpu_baseline"] = with_host({"value": 1.0 / dt, "unit": "chromosomes/s", "cores": 1, "kind": "port",
                                             "sample": f"oracle/hichap_ref.two_step_correction (vectorised NumPy) "
                                                       f"on the same chromosome: {dt:.2f} s"})
        print(json.dumps(out), flush=True)


def _dense_pair_device(N, gen, rng, A=60.0, drop_rows=0):
    """synth.dense_chrom + synth.haplotype_pair on the device (torch Poisson /
    binomial draws; the bin profile from synth.bin_profile): T, M, P as int64
    N x N device tensors."""
    import torch
    from hichap_master_amd import synth
    s, v, _ = synth.bin_profile(N, rng, 0.02, (5, 15))
    s = torch.from_numpy(np.asarray(s, np.float64)).cuda()
    v = torch.from_numpy(np.asarray(v, np.float64)).cuda()
    i = torch.arange(N, device="cuda", dtype=torch.float64)
    lam = A * ((i[:, None] - i[None, :]).abs() + 1.0) ** -1.08
    lam *= (1.0 + 0.3 * s[:, None] * s[None, :]) * v[:, None] * v[None, :]
    up = torch.poisson(torch.triu(lam), generator=gen)
    del lam
    TM = torch.triu(up) + torch.triu(up, 1).T
    del up
    base = torch.binomial(TM, torch.full_like(TM, 0.4), generator=gen)
    MM = torch.binomial(base, torch.full_like(base, 0.5), generator=gen)
    PM = base - MM
    del base
    for X in (MM, PM):
        X -= torch.binomial(torch.triu(X, 1), torch.full_like(X, 0.15), generator=gen)
        if drop_rows:
            rows = torch.from_numpy(rng.choice(N, size=drop_rows, replace=False)).cuda()
            X[rows, :] = torch.binomial(X[rows, :], torch.full_like(X[rows, :], 0.02), generator=gen)
            X[:, rows] = torch.binomial(X[:, rows], torch.full_like(X[:, rows], 0.02), generator=gen)
    return tuple(X.to(torch.int64).contiguous() for X in (TM, MM, PM))


def run_twostep_genome(args, world, rank, local):
    """IntraChromMatrixCorrection (matrixBuilding.py:1026-1041, :1607-1614)
    over a whole localRes set: hg19 chromosomes 1-22 + X at 40 kb (HiCHap's
    default chroms ['#', 'X'] and localRes), synthetic T / imputed M, P on the
    device.  A step = every chromosome's two-step correction in one
    hh_twostep_batch call (every pass of every chromosome in one shared
    launch).  Also timed: the same chromosomes one TwoStepCorrection call
    after the other."""
    import torch
    from hichap_master_amd import matrixBuilding as mb, synth
    names = [str(c) for c in range(1, 23)] + ["X"]
    Ns = synth.chrom_bins([synth.HG19[c] for c in names], 40000)
    gen = torch.Generator(device="cuda").manual_seed(20201025)
    rng = np.random.default_rng(20201025)
    tra, hap = {}, {}
    for c, N in zip(names, Ns):
        T, M, P = _dense_pair_device(int(N), gen, rng, drop_rows=max(1, int(N) // 50))
        tra[c], hap["M" + c], hap["P" + c] = T, M, P
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        mb.IntraChromMatrixCorrection(tra, hap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = mb.IntraChromMatrixCorrection(tra, hap)
        del out
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / args.steps
    # one chromosome after the other (the per-call path)
    # (--main-only, the PMC passes: skipped, so every batch dispatch in the
    # profile is a whole-genome step's)
    ks = 0 if args.main_only else max(1, min(3, args.steps))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(ks):
        for c in names:
            mb.TwoStepCorrection(tra[c], hap["M" + c], hap["P" + c])
    torch.cuda.synchronize()
    seq = (time.perf_counter() - t1) / ks if ks else None
    sq = float(sum(int(N) ** 2 for N in Ns))
    alg = 40.0 * sq  # 3 int64 reads + 2 fp64 writes per element
    if rank == 0:
        out = {"metric": "IntraChromMatrixCorrection (TwoStepCorrection per chromosome), hg19 1-22 + X at 40 kb",
               "value": 1.0 / step, "unit": "genomes/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": 1000.0 * step, "higher_is_better": True, "scaling": "replicas", "vs_baseline": None,
               "dtype": "int64 in, f64 out", "data": "synthetic (device Poisson / binomial draws, synth model)",
               "config": {"workload": "twostep-hg19-40kb-genome", "chromosomes": len(names),
                          "bins": int(sum(int(N) for N in Ns)), "sum_N2": sq,
                          "launches": "shared per pass" if mb.TWOSTEP_STREAMS == 0 else f"{mb.TWOSTEP_STREAMS} streams"},
               "roofline": {"bound": "hbm", "kernel": "hh_twostep_batch (shared launches: k_rowstats_b, k_ts_gapdef_b, "
                                                       "k_ts_alpha_b, then the symmetrisation passes k_sv_*_b of every "
                                                       "chromosome's MM and PM)",
                            "achieved": alg / step / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": alg / step / 1e9 / PEAK_HBM_GBS, "traffic": None, "alg_bytes_per_launch": alg,
                            "note": "40 B per matrix element (3 int64 reads + 2 fp64 writes), the whole genome per step"},
               "sequential_ms": None if args.main_only else 1000.0 * seq,
               "note": "sequential_ms: the same 23 chromosomes as one TwoStepCorrection call each"}
        tr, tr_src = twostep_pmc_traffic("twostep_genome", {"workload": "twostep-hg19-40kb-genome",
                                                            "bins": int(sum(int(N) for N in Ns)), "sum_N2": sq})
        if tr:
            out["roofline"].update(traffic=tr, traffic_source=tr_src, traffic_GBps=tr / step / 1e9,
                                   traffic_frac=tr / step / 1e9 / PEAK_HBM_GBS,
                                   traffic_note="2 x FETCH_SIZE + WRITE_SIZE of the batch kernels per genome")
        if not args.no_cpu:
            from oracle import hichap_ref
            k = names.index("21")
            T, M, P = (X.cpu().numpy() for X in (tra["21"], hap["M21"], hap["P21"]))
            t = time.perf_counter()
            hichap_ref.two_step_correction(T, M, P)
            dt = time.perf_counter() - t
            est = dt * sq / float(int(Ns[k]) ** 2)
            out["cpu_baseline"] = with_host({"value": 1.0 / est, "unit": "genomes/s (extrapolated by sum N^2)",
                                             "cores": 1, "kind": "port",
                                             "sample": f"oracle/hichap_ref.two_step_correction (vectorised NumPy) on "
                                                       f"chr21 (N = {int(Ns[k])}): {dt:.3f} s, x sum N^2 / N21^2"})
        print(json.dumps(out), flush=True)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count():
    """GPUs this process may use, counted WITHOUT loading the HIP runtime (the
    launcher must not initialise HIP before its ranks start, and torch loads
    libamdhip64 on import): the KFD topology in sysfs (nodes whose
    ``gfx_target_version`` is nonzero; ``HH_KFD_TOPOLOGY`` overrides the path
    for tests), narrowed by ROCR_ / HIP_ / CUDA_VISIBLE_DEVICES.  Where the
    topology cannot be read, a child process counts through torch."""
    import glob
    import subprocess
    root = os.environ.get("HH_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology/nodes")
    nodes = glob.glob(os.path.join(root, "*", "properties"))
    n = 0
    for path in nodes:
        try:
            with open(path) as f:
                for line in f:
                    key, _, val = line.strip().partition(" ")
                    if key == "gfx_target_version":
                        n += int(val) != 0
                        break
        except (OSError, ValueError):
            continue
    if not nodes:
        p = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=600)
        try:
            n = int(p.stdout.strip().splitlines()[-1])
        except (ValueError, IndexError):
            n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(n, argv):
    """``bench.py --gpus N`` without a launcher: start N child ranks (one
    process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
    environment, as torch.distributed.run sets them) and return the exit
    status.  Runs before anything touches the GPU in this process: counting
    devices does not initialise HIP on this image, and the children bind their
    own device.  Rank 0's stdout (the JSON line) passes through; if any rank
    fails, the others are stopped (by PID) and the status is non-zero.
    ``HH_DEVICE`` set = a path check with every rank on that one device
    (``HH_DIST_BACKEND=gloo``), so no device count is required."""
    import subprocess
    if "HH_DEVICE" not in os.environ:
        ndev = visible_gpu_count()
        if ndev < n:
            print(f"[bench] --gpus {n} needs {n} visible GPUs, this node has {ndev}; refusing to report "
                  f"n_gpus={n} from fewer devices (set HH_DEVICE=<dev> HH_DIST_BACKEND=gloo for a one-device "
                  f"path check)", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"[bench] rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) to run on; without a launcher's WORLD_SIZE, bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--nnz", type=float, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--main-only", action="store_true",
                    help="TwoStep lines: time the step only, no side measurements (the PMC passes)")
    ap.add_argument("--pairs", type=float, default=2e8, help="pairs per rank for --config pairs")
    ap.add_argument("--iters", type=int, default=200, help="ICE iteration cap for --config dropin / e2e")
    ap.add_argument("--fixed-iters", action="store_true", help="dropin: tol 0 (exactly --iters iterations)")
    ap.add_argument("--res", type=int, default=10000, help="whole-genome resolution for --config e2e")
    ap.add_argument("--gw-t", type=float, default=1.5e9, help="--config gw: T upper pixels")
    ap.add_argument("--gw-h", type=float, default=1.5e9, help="--config gw: H ordered cells")
    ap.add_argument("--sharded", action="store_true",
                    help="use the multi-GPU (all-gather) driver even at N=1 (path check)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if (args.gpus or 1) > 1:  # no launcher: start the ranks ourselves (no GPU call in this process)
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif args.gpus is not None and int(env_world) != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={env_world}: the launcher and the flag disagree",
              file=sys.stderr, flush=True)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # path checks on a 1-GPU box only: every rank on one device, gloo exchange
    local = int(os.environ.get("HH_DEVICE", local))
    backend = os.environ.get("HH_DIST_BACKEND", "nccl")
    import torch
    torch.cuda.set_device(local)
    from hichap_master_amd import _lib, dist, ice
    _lib.load()
    _lib.call("hh_set_device", local)
    for key in ("pca_p", "pca_method", "pca_debug", "build_debug"):  # eigensolver / build-trace knobs (measurement)
        if os.environ.get("HH_" + key.upper()):
            _lib.call("hh_tune", key.encode(), int(os.environ["HH_" + key.upper()]))
    if world > 1 or args.sharded:
        import torch.distributed as tdist
        if "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0", WORLD_SIZE="1")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)

    if args.config in ("c5", "pairs", "loops", "dropin", "e2e", "gw", "twostep", "twostep_genome"):
        {"c5": run_c5, "pairs": run_pairs, "loops": run_loops, "dropin": run_dropin,
         "e2e": run_e2e, "gw": run_gw, "twostep": run_twostep,
         "twostep_genome": run_twostep_genome}[args.config](args, world, rank, local)
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return
    sizes, kw, label, target, tf = config(args.config, args.nnz)
    n = int(np.sum(sizes))
    t0 = time.perf_counter()
    rc, ru = ice.synth_row_counts(sizes, **kw)
    rank_rows = dist.partition_rows(rc, world)
    m = ice.ContactMatrix.synthetic(sizes, row_range=(rank_rows[rank], rank_rows[rank + 1]), **kw)
    opts = ice.IceOptions(tol=0.0, max_iters=1 << 30, cis_only=bool(kw.get("cis_only")))
    st = ice.IceState(m, opts)
    stream = torch.cuda.current_stream().cuda_stream
    if world > 1:
        # (shards below 8 GB of payload sweep on one stream, the library
        # default: C4 at N=8 has 1.6-1.9 GB per shard)
        if not os.environ.get("HH_NO_REFINE"):
            # setup, untimed: one measured refinement of the row partition
            # (payload bytes mis-price rows whose bytes sweep at different rates)
            def costs():
                ms = torch.tensor([measure_shard_sweep_ms(st, rank_rows[rank + 1] - rank_rows[rank], stream)],
                                  dtype=torch.float64, device="cuda")
                allms = [torch.zeros_like(ms) for _ in range(world)]
                torch.distributed.all_gather(allms, ms)
                return [float(x.item()) for x in allms]

            def rebuild(rr):
                nonlocal m, st, rank_rows
                st.close()
                m.close()
                rank_rows = rr
                m = ice.ContactMatrix.synthetic(sizes, row_range=(rank_rows[rank], rank_rows[rank + 1]), **kw)
                st = ice.IceState(m, opts)

            cost = costs()
            rr0 = rank_rows
            rr2 = dist.partition_rows(dist.refine_weights(rc, rank_rows, cost), world)
            if not np.array_equal(rr2, rank_rows):
                rebuild(rr2)
                if max(costs()) > max(cost):  # measured worse (noise): keep the payload partition
                    rebuild(rr0)
    gen_s = time.perf_counter() - t0
    inf = m.info()
    nnz_total = int(ru.sum())

    def barrier():
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize()

    dist_impl = "single"
    if world == 1 and not args.sharded:
        # filters (untimed), then warmup + timed iterations in one C++ loop each
        st.marg_local(0, None, stream); st.filter_nnz(stream)
        st.marg_local(1, None, stream); st.filter_count_mad(stream)
        # the timed loop without per-sweep HIP events (their markers cost the
        # small matrices' iterations microseconds); the sweep time for the
        # roofline from a few more iterations with the events on, after it
        _lib.call("hh_tune", b"iter_events", 0)
        st.run(args.warmup, stream)
        barrier()
        t_start = time.perf_counter()
        st.run(args.steps, stream)
        barrier()
        elapsed = time.perf_counter() - t_start
        _lib.call("hh_tune", b"iter_events", 1)
        st.run(max(1, min(args.steps, 5)), stream)
        sweep_ms, launches, iter_ms = st.last_timing()
    else:
        # the iteration loop in C++ (hh_ice_run_sharded) with the library's
        # own RCCL communicator; HH_DIST_IMPL=torch keeps the Python loop with
        # torch.distributed's all-gather (also the fallback if RCCL init fails)
        impl = os.environ.get("HH_DIST_IMPL", "capi")
        cx = None
        if impl == "capi":
            try:
                cx = dist.CapiExchange(rank_rows, world, rank, backend=backend)
            except Exception as e:  # noqa: BLE001
                print(f"[bench] C-ABI exchange unavailable ({e}); using torch.distributed", file=sys.stderr)
                impl = "torch"
        if impl == "capi":
            run = lambda k: dist.iterate_capi(st, cx, k, stream)
            dist.filters_capi(st, cx, stream)
        else:
            ex = dist.Exchange(rank_rows, torch.device("cuda", local))
            run = lambda k: dist.iterate(st, ex, k)
            dist.run_filters(st, ex)
        run(args.warmup)
        barrier()
        t_start = time.perf_counter()
        run(args.steps)
        barrier()
        elapsed = time.perf_counter() - t_start
        # sweep-kernel timing: a few more iterations with the HIP-event
        # registry on (after the timed region; events cost ~µs per launch)
        n_prof = max(1, min(args.steps, 5))
        _lib.call("hh_ktime_reset")
        _lib.call("hh_ktime_enable", 1)
        t_it = time.perf_counter()
        run(n_prof)
        torch.cuda.synchronize()
        iter_ms = 1000.0 * (time.perf_counter() - t_it)
        _lib.call("hh_ktime_enable", 0)
        sweep_ms, launches = _lib.ktime("ice_sweep")
        _lib.call("hh_ktime_reset")
        dist_impl = impl
        if cx is not None:
            cx.close()
    tad = tad_scan_bench(m, st, stream) if args.config == "c2" and world == 1 and not args.sharded else None
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(tt.item())

    # the slowest rank's sweep bounds the iteration: report its shard
    # a shard stores both triangles of its rows: its share of the 12 B/pixel
    # algorithmic traffic is half its stored entries (= nnz_upper at N=1)
    shard_pix = float(inf["nnz_upper"]) if world == 1 else 0.5 * float(inf["n_entries"])
    # bytes the state's sweep kernels read: tiles + row pointers + the bands
    # (their upper halves only with the upper-band sweep)
    shard = torch.tensor([sweep_ms / max(launches, 1), shard_pix, float(st.swept_bytes())],
                         dtype=torch.float64, device="cuda")
    if torch.distributed.is_initialized():
        allsh = [torch.zeros_like(shard) for _ in range(world)]
        torch.distributed.all_gather(allsh, shard)
        shard = max(allsh, key=lambda t: float(t[0]))
    shard_sweep_ms, shard_nnz, shard_real = (float(x) for x in shard.cpu())

    if rank == 0:
        its = args.steps / elapsed
        out = {
            "metric": "ICE iterations/sec on 10 kb whole-genome matrix (also nnz*iters/sec)",
            "value": its, "unit": "ICE iterations/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d) model generated in HBM; no real Hi-C data offline)",
            "nnz_iters_per_s": nnz_total * its,
            "config": {"workload": label, "n_bins": n, "nnz_upper": nnz_total,
                       **({"config_note": "trans fraction 0.85, not SURVEY 8(d)'s ~0.2: hg19 at 40 kb has only "
                                          "1.42e8 cis pixels, so BASELINE C3's 8e8 nnz needs ~85 % trans"}
                          if args.config == "c3" else {}),
                       **({"config_note": "haploid traditional T matrix (303 641 bins): the one HiCHap balances "
                                          "genome-wide at 10 kb, matrixBuilding.py:1536-1538; trans fraction 0.6: "
                                          "it has only 2.36e9 cis pairs, so 5e9 pixels need >= 53 % trans"}
                          if args.config == "c4h" else {}),
                       **({"config_note": "cooler balance --cis-only (matrixBuilding.py:713): every chromosome "
                                          "its own ICE group in one matrix, all iterated (tol 0), one launch "
                                          "chain per iteration for the whole genome", "cis_only": True}
                          if args.config == "cis" else {}),
                       "trans_fraction_target": tf, "resolution_bp": 40000 if args.config in ("c1", "c3") else 10000,
                       "parallelism": f"rows sharded x{world} (measured-cost partition), {'RCCL' if backend == 'nccl' else backend} all-gather of marginals, loop in {'C++ (hh_ice_run_sharded)' if dist_impl == 'capi' else 'Python'}" if world > 1
                       else "single GPU", "generate_s": round(gen_s, 2),
                       "entries_stored": inf["n_entries"], "slots_u32": inf["n_slots"],
                       "slots_u16": inf["n_slots_narrow"], "payload_bytes": inf["payload_bytes"],
                       "tiles": inf["n_tiles"], "units": inf["n_units"],
                       "hbm_bytes_matrix": inf["device_bytes"]},
        }
        traffic, meta, traffic_src = (pmc_traffic({"n_bins": n, "nnz_upper": nnz_total}, line=args.config)
                                      if args.config in PMC_SOURCES else (None, None, None))
        if launches:
            # per launch on the slowest rank (= the whole matrix at N=1)
            sweep_avg = shard_sweep_ms / 1000.0
            alg_gbps = ALG_BYTES_PER_PIXEL * shard_nnz / sweep_avg / 1e9
            # bytes the layout actually streams: entries (uint16 + uint32) +
            # both segments' row pointers (the b staging shows up in traffic)
            real_b = shard_real
            if traffic and world > 1:
                # the PMC summary is of the whole matrix: scale its
                # traffic-per-payload-byte ratio to this shard's payload
                full_real = (meta or {}).get("real_bytes_per_sweep")
                traffic = traffic / full_real * real_b if full_real else None
                traffic_src = f"{traffic_src} (scaled by shard payload)" if traffic else None
            phys = traffic if traffic else real_b
            achieved = phys / sweep_avg / 1e9
            pb = inf["payload_bytes"]
            ub = st.swept_bytes() < pb  # the upper-band sweep reads half the bands
            band_k = ("k_sweep_ubands (upper halves of the uint8 + 4-bit bands, each count to its row and column)"
                      if ub else "k_sweep_bands (uint8 + 2 x 4-bit segments)")
            out["roofline"] = {"bound": "hbm", "kernel": (f"ice sweep span: k_sweep_flatw | k_sweep_tiled | {band_k} on three streams"
                                         if pb >= (8 << 30) else
                                         f"ice sweep: k_sweep_tiled, k_sweep_flatw, {band_k} on one stream"
                                         if pb >= (1 << 30) else
                                         "ice sweep: k_sweep_all (tiled + band + flat bodies in one launch)")
                               + " (HIP events around the sweep; rocprof per-sweep span: tools/sweep_span.py)",
                               "achieved": achieved,
                               "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                               "bytes_per_launch": phys,
                               "bytes_source": "PMC traffic" if traffic else "layout payload (no PMC summary)",
                               "traffic": traffic,
                               "traffic_source": traffic_src,
                               "traffic_profile_commit": (meta or {}).get("commit"),
                               "real_bytes_per_launch": real_b,
                               "real_GBps": real_b / sweep_avg / 1e9,
                               "real_frac": real_b / sweep_avg / 1e9 / PEAK_HBM_GBS,
                               "alg_effective_GBps": alg_gbps,
                               "alg_bytes_per_launch": ALG_BYTES_PER_PIXEL * shard_nnz,
                               "sweep_ms_avg": sweep_avg * 1000.0,
                               "iter_ms_avg": iter_ms / launches,
                               "per_rank": "slowest rank's shard" if world > 1 else "whole matrix",
                               "shard_nnz_upper": shard_nnz,
                               "note": "achieved / frac = physical HBM bytes per sweep (PMC traffic, else the "
                                       "layout's payload) / sweep time; alg_effective_GBps = SURVEY 8(d)'s "
                                       "12 B/pixel / sweep time (> peak: the layout streams ~3 B/pixel, DESIGN.md 3)"}
        if tad is not None:
            out["tad_scan"] = tad
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = with_host(cpu_baseline(sizes, kw, rc, nnz_total, label))
            # vs_baseline stays null (BASELINE.md publishes no number for this
            # metric); the ratio to the measured CPU baseline is reported here
            out["vs_cpu_baseline"] = its / out["cpu_baseline"]["value"]
        print(json.dumps(out), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
