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

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2]
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
ALG_BYTES_PER_PIXEL = 12.0  # int32 bin1 + int32 bin2 + fp32 count


def config(name, nnz=None):
    from hichap_master_amd import synth
    if name == "c4":
        sizes = synth.genome_bins(10000, diploid=True)
        target, tf, label = nnz or 5e9, 0.2, "hg19-10kb-diploid-wholegenome"
    elif name == "c2":
        sizes = [synth.chrom_bins([synth.HG19["1"]], 10000)[0]]
        target, tf, label = nnz or 5e7, 0.0, "hg19-chr1-10kb"
    else:
        raise SystemExit(f"unknown config {name}")
    A, td = synth.calibrate(sizes, target, tf)
    return sizes, dict(A=A, trans_density=td, comp_block=200, seed=20201015), label, target, tf


def pmc_traffic(kernel="k_sweep_tiled"):
    """HBM bytes per launch of the sweep kernel from the committed rocprofv3
    PMC summary of this same command (tools/pmc_summary.py), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_c4_pmc.json")))
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    for k, v in data.items():
        if kernel in k:
            return v["traffic_bytes"], os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_baseline(sizes, kw, rc, nnz_total, budget_s=12.0):
    """Oracle (NumPy, cooler's bincount sweep) timed on the host on a bounded
    sample: the upper-triangle pixels of the first rows of the same matrix."""
    from hichap_master_amd import ice
    from oracle import ice_ref
    n = int(np.sum(sizes))
    per_row = max(nnz_total / n, 1.0)
    rows = int(min(n, max(64, 2.5e7 / per_row)))
    rows = min(n, (rows + 255) // 256 * 256)
    m = ice.ContactMatrix.synthetic(sizes, row_range=(0, rows), **kw)
    b1, b2, c = m.export_upper()
    m.close()
    t0 = time.perf_counter()
    iters = 0
    while True:
        ice_ref.sweep_rate(b1, b2, c, n, 1)
        iters += 1
        if time.perf_counter() - t0 > budget_s or iters >= 50:
            break
    dt = time.perf_counter() - t0
    pix_rate = b1.size * iters / dt
    return {"value": pix_rate / nnz_total, "unit": "ICE iterations/s (whole C4 matrix, extrapolated)",
            "cores": 1, "kind": "port",
            "sample": f"oracle/ice_ref.sweep_rate (numpy bincount, cooler restatement) on the "
                      f"{b1.size} upper pixels of rows [0,{rows}) of the same matrix, {iters} sweeps "
                      f"in {dt:.1f}s = {pix_rate:.3g} pixel-iters/s",
            "pixel_iters_per_s": pix_rate}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--nnz", type=float, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sharded", action="store_true",
                    help="use the multi-GPU (all-gather) driver even at N=1 (path check)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    from hichap_master_amd import _lib, dist, ice
    _lib.load()
    _lib.call("hh_set_device", local)
    if world > 1 or args.sharded:
        import torch.distributed as tdist
        if "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0", WORLD_SIZE="1")
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))

    sizes, kw, label, target, tf = config(args.config, args.nnz)
    n = int(np.sum(sizes))
    t0 = time.perf_counter()
    rc, ru = ice.synth_row_counts(sizes, **kw)
    rank_rows = dist.partition_rows(rc, world)
    m = ice.ContactMatrix.synthetic(sizes, row_range=(rank_rows[rank], rank_rows[rank + 1]), **kw)
    gen_s = time.perf_counter() - t0
    inf = m.info()
    nnz_total = int(ru.sum())
    opts = ice.IceOptions(tol=0.0, max_iters=1 << 30)
    st = ice.IceState(m, opts)
    stream = torch.cuda.current_stream().cuda_stream

    def barrier():
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        torch.cuda.synchronize()

    if world == 1 and not args.sharded:
        # filters (untimed), then warmup + timed iterations in one C++ loop each
        st.marg_local(0, None, stream); st.filter_nnz(stream)
        st.marg_local(1, None, stream); st.filter_count_mad(stream)
        st.run(args.warmup, stream)
        barrier()
        t_start = time.perf_counter()
        st.run(args.steps, stream)
        barrier()
        elapsed = time.perf_counter() - t_start
        sweep_ms, launches, iter_ms = st.last_timing()
    else:
        ex = dist.Exchange(rank_rows, torch.device("cuda", local))
        dist.run_filters(st, ex)
        dist.iterate(st, ex, args.warmup)
        barrier()
        t_start = time.perf_counter()
        dist.iterate(st, ex, args.steps)
        barrier()
        elapsed = time.perf_counter() - t_start
        sweep_ms, launches, iter_ms = float("nan"), 0, float("nan")
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(tt.item())

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
                       "trans_fraction_target": tf, "resolution_bp": 10000 if args.config != "c1" else 40000,
                       "parallelism": f"rows sharded x{world}, RCCL all-gather of marginals" if world > 1
                       else "single GPU", "generate_s": round(gen_s, 2),
                       "entries_stored": inf["n_entries"], "slots": inf["n_slots"],
                       "tiles": inf["n_tiles"], "units": inf["n_units"],
                       "hbm_bytes_matrix": inf["device_bytes"]},
        }
        traffic, traffic_src = (pmc_traffic() if args.config == "c4" and args.nnz is None
                                else (None, None))
        if launches:
            sweep_avg = sweep_ms / launches / 1000.0
            achieved = ALG_BYTES_PER_PIXEL * inf["nnz_upper"] / sweep_avg / 1e9
            out["roofline"] = {"bound": "hbm", "kernel": "k_sweep_tiled", "achieved": achieved,
                               "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                               "traffic": traffic,
                               "traffic_source": traffic_src,
                               "real_bytes_per_launch": 4.0 * inf["n_slots"] + 4.0 * 257 * inf["n_tiles"],
                               "sweep_ms_avg": sweep_avg * 1000.0,
                               "iter_ms_avg": iter_ms / launches}
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(sizes, kw, rc, nnz_total)
        print(json.dumps(out), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
