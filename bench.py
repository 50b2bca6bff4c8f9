#!/usr/bin/env python3
"""Benchmark: the fused S10 suite over a synthetic 1e9-row Item table per GPU.

One step = one pass of the hot path over the table resident in HBM: reset the aggregation state,
the fused scan of every record batch in ONE launch (+ the finalize launch), the state read-back
and, with N > 1 ranks, the exchange step on the device (distributed.exchange_states: counters in
one RCCL all-reduce SUM, extremes and HLL registers in one all-reduce MAX, the fp64 moments
all-gathered and merged in rank order by a kernel).  Rows are sharded across ranks with no data-path collective, so
per-GPU work is fixed (weak scaling); `value` = rows of all ranks / max-over-ranks step time.

Output: ONE JSON line (rank 0).  `roofline.achieved` = algorithmic bytes of the suite (the distinct
buffers it must read) / the average duration of the scan launch measured with HIP
events on the engine's stream over the timed region; `cpu_baseline` = the C restatement of Spark
2.2 deequ semantics (oracle/oracle.c, "port") timed on this host's cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rows/sec + achieved HBM GB/s, fused 10-analyzer suite on 1B rows, 1/2/4/8 GPUs"
PEAK_HBM = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md:36)


def s10_suite():
    from deequ_amd.analyzers import (Completeness, Compliance, Maximum, Mean, Minimum, Size,
                                     StandardDeviation, Sum)
    return [Size(), Completeness("id"), Completeness("name"),
            Compliance("numViews is non-negative", "numViews >= 0"),
            Compliance("priority contained in high,low",
                       "priority IS NULL OR priority IN ('high','low')"),
            Sum("numViews"), Mean("numViews"), StandardDeviation("numViews"),
            Minimum("numViews"), Maximum("numViews")]


def algorithmic_bytes(table) -> int:
    """Distinct buffers S10 must read: 4 validity bitmaps, numViews values, priority offsets and
    bytes."""
    total = 0
    for b in table.batches:
        n = b["id"].length
        total += 4 * ((n + 7) // 8)              # id/name/priority/numViews validity
        total += 8 * n                           # numViews values
        total += 4 * (n + 1)                     # priority offsets
        total += int(b["priority"].values[n].item())  # priority bytes
    return total


def available_cpus() -> tuple:
    """(CPUs this process may run on, CPUs of the host): the affinity mask, capped by a cgroup v2
    `cpu.max` quota when one is set (a GPU box's share of a larger host)."""
    host = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n, host


def cpu_baseline(rows: int, seed: int, min_seconds: float = 10.0):
    """oracle/oracle.c S10 as ONE pass per partition (the reference's single Spark job, local[T]
    with T = every CPU this process may use) on a bounded sample."""
    from deequ_amd.synth import item_buffers_numpy
    from oracle import c_oracle as C
    threads, host = available_cpus()
    buf = item_buffers_numpy(rows, seed)
    n = buf["n"]
    res = C.s10_fused(buf, threads=threads)
    assert res.rows == n
    reps, t0 = 0, time.perf_counter()
    while True:
        C.s10_fused(buf, threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds or reps >= 5000:
            break
    return {"value": reps * n / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"S10 over {n} synthetic Item rows x {reps} passes ({el:.1f} s): one fused "
                      f"pass per partition, CPU restatement of Spark 2.2 deequ semantics "
                      f"(oracle/oracle.c, OpenMP, {threads} threads = Spark local[{threads}], every "
                      f"CPU this process may use; the host has {host}) -- not Spark"}


def h2d_inclusive(plan, state, seed: int, batch_rows: int = 1 << 24, passes: int = 8):
    """The same S10 scan fed from HOST Arrow-layout buffers through the columnar loader
    (dq_scan_host: pinned staging, DMA on the loader's stream overlapping the previous batch's
    scan; only the buffers the plan reads cross the link).  Two distinct host batches, scanned
    `passes` times in turn, timed from the first staging to the state read-back."""
    import numpy as np

    from deequ_amd import _native as N
    from deequ_amd.loader import HostColumn, HostLoader
    from deequ_amd.runners.engine import read_row
    from deequ_amd.synth import item_buffers_numpy
    batches = []
    for k in range(2):
        b = item_buffers_numpy(batch_rows, seed, start=k * batch_rows)
        n = b["n"]
        dummy8, dummy4, dummyb = np.zeros(2, np.int64), np.zeros(4, np.int32), np.zeros(16, np.uint8)
        cols = {  # id / name: Completeness reads their validity alone (nothing else is staged)
            "id": HostColumn(N.INT64, n, b["id_valid"], dummy8),
            "name": HostColumn(N.UTF8, n, b["name_valid"], dummy4, dummyb),
            "priority": HostColumn(N.UTF8, n, b["priority_valid"], b["priority_offsets"],
                                   b["priority_data"]),
            "numViews": HostColumn(N.INT64, n, b["numViews_valid"], b["numViews"]),
        }
        batches.append(cols)
    nb = lambda m: (m + 7) // 8  # noqa: E731
    link_bytes = sum(4 * nb(c["id"].length) + 4 * (c["id"].length + 1) +
                     int(c["priority"].values[c["id"].length]) + 8 * c["id"].length
                     for c in batches) * passes // 2
    loader = HostLoader(0)
    N.check(N.lib.dq_state_reset(state))
    loader.scan(plan, state, batches[0])  # warm the pinned staging buffers
    read_row(plan, state)
    N.check(N.lib.dq_state_reset(state))
    t0 = time.perf_counter()
    for i in range(passes):
        loader.scan(plan, state, batches[i % 2])
    row = read_row(plan, state)
    el = time.perf_counter() - t0
    assert row[0] == passes * batch_rows
    return {"value": passes * batch_rows / el, "unit": "rows/s", "rows": passes * batch_rows,
            "link_bytes": link_bytes, "link_GBps": link_bytes / el / 1e9,
            "path": "host Arrow buffers -> dq_scan_host (pinned staging + DMA overlapped with the "
                    "scan); only the buffers the plan reads cross the link"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1_000_000_000, help="rows per GPU")
    ap.add_argument("--batch-rows", type=int, default=1 << 26)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cpu-rows", type=int, default=20_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="skip the host-fed (PCIe) measurement")
    ap.add_argument("--workloads", default="c3,c4,c5",
                    help="after the S10 leg (N=1 only): configs[2] (c3), configs[3] (c4) and "
                         "configs[4] (c5) timed at their stated sizes; '' skips them")
    ap.add_argument("--workload-budget-s", type=float, default=360.0,
                    help="wall-clock budget of the whole run: a workload is skipped (and says so) "
                         "once it would start past this many seconds")
    args = ap.parse_args()
    t_start = time.perf_counter()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run as a CHILD process, before this
        # process touches the GPU, and exit with its code
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
               str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and int(os.environ.get("RANK", "0")) == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)",
              file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    device = f"cuda:{local}"
    torch.cuda.set_device(local)

    from deequ_amd import _native as N
    from deequ_amd.analyzers.base import AggSpec  # noqa: F401
    from deequ_amd.distributed import exchange_states
    from deequ_amd.runners.engine import get_plan, read_row, scan_into
    from deequ_amd.synth import item_table_device

    table = item_table_device(args.rows, seed=args.seed, batch_rows=args.batch_rows,
                              device=device, start=rank * args.rows)
    suite = s10_suite()
    specs = [s for a in suite for s in a.aggregation_functions()]
    plan = get_plan(table.schema, specs)
    state = plan.state(local)
    stream = torch.cuda.current_stream(device)
    sh = ctypes.c_void_p(stream.cuda_stream)
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def step(i=None):
        N.check(N.lib.dq_state_reset(state))
        if i is not None:
            ev0[i].record(stream)
        scan_into(table, plan, state, sh)
        if i is not None:
            ev1[i].record(stream)
        if world > 1:  # SUM / MAX all-reduces + gathered moments merged on the device
            return exchange_states(plan, state, device)
        N.check(N.lib.dq_state_sync(state))
        return read_row(plan, state)

    for _ in range(args.warmup):
        row = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(args.steps):
        row = step(i)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    scan_ms = sum(a.elapsed_time(b) for a, b in zip(ev0, ev1)) / args.steps
    b_alg = algorithmic_bytes(table)
    achieved = b_alg / (scan_ms * 1e-3)

    # sanity: the row must be a valid S10 result
    assert row[0] == args.rows * world or world > 1 or row[0] == args.rows

    traffic, traffic_src = load_traffic(args.rows, b_alg)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": args.rows * world / (elapsed / args.steps),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": "S10 fused suite (Size, Completeness(id), Completeness(name), "
                            "Compliance(numViews >= 0), Compliance(priority IS NULL OR priority IN "
                            "('high','low')), Sum/Mean/StandardDeviation/Minimum/Maximum(numViews)) "
                            "over a synthetic Item table: int64 id/numViews, string name/priority, "
                            "5% nulls (BASELINE.json configs[1])",
                "rows_per_gpu": args.rows,
                "batch_rows": args.batch_rows,
                "parallelism": f"dp{world}",
            },
            "achieved_hbm_gbps": achieved / 1e9,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved / 1e9,
                "peak": PEAK_HBM / 1e9,
                "unit": "GB/s",
                "frac": achieved / PEAK_HBM,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": b_alg,
                "scan_ms": scan_ms,
                "kernel": "dq::scan_mixed_kernel (+ finalize_kernel)",
                "scan_code_object_sha": scan_code_object_hash(),
            },
        }
        if world == 1 and not args.no_h2d:
            out["h2d_inclusive"] = h2d_inclusive(plan, state, args.seed)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_rows, args.seed)
        if world == 1 and args.workloads:
            del table, state, plan
            N.release_cached_memory()
            out["workloads"] = other_workloads(args, t_start)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


WORKLOAD_CONFIG = {"c3": "configs[2]", "c4": "configs[3]", "c5": "configs[4]"}


def other_workloads(args, t_start: float) -> dict:
    """BASELINE.json configs[2]-[4] on this GPU, after the S10 leg and outside its timed region
    (tools/bench_workloads.run_single: each builds its synthetic table at the stated per-GPU size,
    runs untimed warmup steps, then times its steps between two device syncs).  Each record carries
    ms_per_step, algorithmic_bytes and frac (= algorithmic bytes / device time per step / 8 TB/s)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_workloads as W
    from deequ_amd import _native as N
    res = {}
    for wl in [w for w in args.workloads.split(",") if w]:
        key = WORKLOAD_CONFIG[wl]
        if time.perf_counter() - t_start > args.workload_budget_s:
            res[key] = {"workload": wl, "skipped": f"past the {args.workload_budget_s:.0f} s budget"}
            continue
        steps = min(args.steps, 5) if wl == "c5" else args.steps
        t0 = time.perf_counter()
        # two untimed steps always: a reused table's buffers reach their size in its second step
        # (configs[2]'s priority table grows its chunk region then, ~17 GB of copies once)
        r = W.run_single(wl, W.DEFAULT_ROWS[wl], steps, 2, args.batch_rows)
        r["wall_s_incl_table_build"] = time.perf_counter() - t0
        res[key] = r
        N.release_cached_memory()
        print(f"bench.py: {key} ({wl}) {r['ms_per_step']:.2f} ms/step, frac "
              f"{r['frac']:.4f}", file=sys.stderr, flush=True)
    return res


def scan_code_object_hash() -> str:
    """sha256 (16 hex digits) of the gfx950 code object that holds dq::scan_mixed_kernel, read from
    the clang offload bundles in libdeequ_amd.so's .hip_fatbin section.  Each HIP translation unit
    is its own bundle, so this is exactly scan.hip's device code as built: host-only edits (a
    prototype in kernels.h) leave it unchanged, any change to the scan kernels' ISA changes it.  A
    PMC traffic figure only describes the build whose code object hashes the same."""
    import hashlib
    import struct
    from deequ_amd import _native
    data = open(_native.LIB_PATH, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    while pos >= 0:
        p = pos + len(magic)
        (entries,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(entries):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            code = data[pos + off:pos + off + size]
            if "gfx950" in triple and b"scan_mixed_kernel" in code:
                return hashlib.sha256(code).hexdigest()[:16]
        pos = data.find(magic, pos + 1)
    raise RuntimeError("no gfx950 code object with scan_mixed_kernel in " + _native.LIB_PATH)


def load_traffic(rows: int, b_alg: int):
    """(HBM bytes per scan launch, source) from the committed rocprofv3 PMC passes
    (profiles/traffic_s10.json) when they were recorded for this workload size AND this build of
    the scan kernel (its gfx950 code object's hash); else (None, why)."""
    path = os.path.join(ROOT, "profiles", "traffic_s10.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, "no profiles/traffic_s10.json"
    if int(d.get("rows_per_gpu", -1)) != rows:
        return None, f"profiles/traffic_s10.json is for {d.get('rows_per_gpu')} rows per GPU"
    sha = scan_code_object_hash()
    if d.get("scan_code_object_sha") != sha:
        return None, (f"profiles/traffic_s10.json ({d.get('tag')}) was measured on another build "
                      f"of the scan kernel (code object hash {d.get('scan_code_object_sha')} != "
                      f"{sha})")
    return d["hbm_bytes_per_launch"], (
        f"profiles/traffic_s10.json ({d.get('tag')}, scan.hip gfx950 code object sha256 {sha}): "
        "HBM bytes per scan launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
        "of this command (FETCH_SIZE x 2 on gfx950, KiB units), not this run")


if __name__ == "__main__":
    main()
