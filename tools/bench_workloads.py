#!/usr/bin/env python3
"""Single-GPU measurements of BASELINE.json configs[2] and configs[3] (the default bench.py line is
configs[1], S10).  Not part of the driver's bench contract; the JSON lines land in profiles/.

  c3: Uniqueness + Distinctness + Entropy + Histogram on the high-cardinality int64 `id` (exact
      mode, ~N groups) and the 3-value string `priority` (hashed mode).  One step = the two
      groupings (+ the one aggregation over each frequency table, dq_freq_summarize) and the two
      Histogram group-bys (+ dq_freq_topk(1000) and the bin count), over the table resident in HBM.
      B_alg = key bytes read once per group-by: id validity + values (8.125 B/row);
      priority validity + offsets + bytes (each column's Histogram table serves its grouping, so
      each column is read once).  Partition traffic excluded.
  c4: ApproxCountDistinct(id) (HLL++, P = 9) + Correlation(id, score) on an Item table with an
      fp64 `score` column.  One step = the fused scan (HLL launch + co-moment launch + finalize).
      B_alg = id validity + values + score validity + values = 16.25 B/row.

  c5: BASELINE configs[4], the full profiling suite: every analyzer on 20 mixed columns (10 numeric,
      10 strings incl. four URL-bearing description columns; deequ_amd.synth.profiling_table_device)
      through AnalysisRunner -- one fused scan (Size, Completeness, Compliance, Sum, Mean,
      StandardDeviation, Minimum, Maximum, Correlation, ApproxCountDistinct, DataType,
      PatternMatch(URL)), one group-by per column for Uniqueness / Distinctness / UniqueValueRatio /
      CountDistinct / Entropy / Histogram (shared except on doubles), the MutualInformation joints,
      and one device sort per ApproxQuantile.  One step = one do_analysis_run.  B_alg = every
      buffer of the table once.

  --gpus N (N > 1): the same workload on N ranks, one per GPU (relaunched under
      torch.distributed.run), weak scaling: --rows per GPU, each rank a row shard of one table,
      through the product's distributed paths; rank 0 prints whole-job rows/s over the slowest
      rank, each rank's ms per step, and each rank's collective bytes per step (run_distributed).
  --cpu-baseline: the C/OpenMP restatement (oracle/oracle.c) timed on a bounded sample.

Usage: python tools/bench_workloads.py c3|c4|c5 [--rows N] [--steps K] [--warmup W] [--gpus N]
       [--cpu-baseline]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["c3", "c4", "c5"])
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch-rows", type=int, default=1 << 26)
    ap.add_argument("--runner", action="store_true", help="c3: time AnalysisRunner itself")
    ap.add_argument("--pyprof", action="store_true", help="cProfile one extra step (stderr)")
    ap.add_argument("--cpu-baseline", action="store_true",
                    help="also time the C/OpenMP restatement (oracle/oracle.c) on a bounded sample")
    ap.add_argument("--cpu-rows", type=int, default=1 << 25, help="rows of that sample")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU (weak scaling: --rows per GPU, row shards of one table)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on cuda:0, collectives over gloo")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: relaunch under torch.distributed.run as a CHILD process, before this
        # process touches the GPU, and exit with its code (as bench.py does)
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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        return run_distributed(args, world, rank, local)
    rows = args.rows or DEFAULT_ROWS[args.workload]
    out = run_single(args.workload, rows, args.steps, args.warmup, args.batch_rows,
                     runner=args.runner, pyprof=args.pyprof, verbose=True,
                     cpu_rows=args.cpu_rows if args.cpu_baseline else None)
    print(json.dumps(out), flush=True)


DEFAULT_ROWS = {"c3": 1_000_000_000, "c4": 1_250_000_000, "c5": 125_000_000}


def run_single(workload: str, rows: int, steps: int, warmup: int, batch_rows: int = 1 << 26,
               runner: bool = False, pyprof: bool = False, verbose: bool = False,
               cpu_rows=None, dev: str = "cuda:0") -> dict:
    """One workload on one GPU: builds its synthetic table in HBM, runs `warmup` untimed steps,
    times `steps` steps (wall clock between two device syncs, and HIP events on the stream per
    step) and returns the JSON record.  bench.py calls it for configs[2]-[4] after its S10 leg."""
    import torch
    from deequ_amd.synth import item_table_device
    if workload == "c5":
        from deequ_amd.synth import profiling_table_device
        # description strings average ~40 B: 2^25-row batches keep int32 offsets in range
        table = profiling_table_device(rows, batch_rows=min(batch_rows, 1 << 25), device=dev)
        torch.cuda.empty_cache()  # the generator's temporaries: the group-bys allocate with hipMalloc
    else:
        table = item_table_device(rows, seed=9, batch_rows=batch_rows, device=dev,
                                  extra=workload == "c4")
    stream = torch.cuda.current_stream(dev)
    e0 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    nb = lambda n: (n + 7) // 8  # noqa: E731

    if workload == "c3":
        from deequ_amd import _native as N
        from deequ_amd.analyzers.grouping import FrequencyTable

        # The group-bys AnalysisRunner plans for this suite (runners/__init__.py): Uniqueness/
        # Distinctness/Entropy share one grouping per column (AnalysisRunner.scala:165-180);
        # Histogram groups with NULL as a group (Histogram.scala:54-69) and takes the device
        # top-1000 + the bin count.  One Histogram-mode table per column serves both (its NULL
        # rows are a group kept apart: the keyed groups are the grouping, dq_freq_summarize_keys,
        # and Histogram folds the NULL group into "NullValue", _fold_null_group).  Tables are
        # created once with their capacity and reset every step (the step still clears, inserts
        # every row, aggregates).  --runner times AnalysisRunner.do_analysis_run itself.
        tables = {"id": (FrequencyTable(["id"], [N.INT64], 0, capacity_hint=rows), N.INT64),
                  "priority": (FrequencyTable(["priority"], [N.UTF8], 0), N.UTF8)}
        from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
        from deequ_amd.analyzers.grouping import KeyedFrequencies, _fold_null_group
        from deequ_amd.runners import AnalysisRunner
        suite = [a for c in ("id", "priority")
                 for a in (Uniqueness([c]), Distinctness([c]), Entropy(c), Histogram(c))]

        def step():
            if runner:
                ctx = AnalysisRunner.do_analysis_run(table, suite)
                return {str(a): ctx.metric(a).value for a in suite}
            out = {}
            for col, (ft, dtype) in tables.items():
                ft.reset()
                for b in table.batches:
                    ft.add([b[col]], null_as_group=True)
                top, bins = _fold_null_group(ft, dtype, 1000)
                out["Histogram(" + col + ")"] = (bins, len(top), top[0])
                s = KeyedFrequencies(ft).summarize()
                out[col] = (s.n_groups, s.n_unique, s.entropy)
            return out
        b_alg = 0
        for b in table.batches:
            m = b["id"].length
            # each group-by reads its key column once
            b_alg += nb(m) + 8 * m + (nb(m) + 4 * (m + 1) + int(b["priority"].values[m].item()))
        kernel = ("dq::freq_phaseA (per batch) + freq_phaseB + freq_phaseC (per table): "
                  "radix-partitioned group-by")
        desc = ("Uniqueness/Distinctness/Entropy grouping + Histogram (top-1000 + bins) on int64 id "
                "(~N groups, exact mode) and string priority (3 groups, hashed mode) over a "
                "synthetic Item table, 5% nulls (BASELINE.json configs[2], 1 GPU)")
        metric_unit = "rows/s"
    elif workload == "c5":
        from deequ_amd import analyzers as A
        from deequ_amd.runners import AnalysisRunner
        suite = c5_suite()

        def step():
            ctx = AnalysisRunner.do_analysis_run(table, suite)
            bad = [(str(a), repr(ctx.metric(a).value.failed)[:300]) for a in suite
                   if not ctx.metric(a).value.is_success]
            if bad:
                raise RuntimeError(f"failed metrics: {bad[:3]}")
            return {"metrics": len(suite),
                    "Histogram(priority_0)": ctx.metric(A.Histogram("priority_0")).value.get().number_of_bins,
                    "PatternMatch(description_0)": ctx.metric(A.PatternMatch("description_0", A.Patterns.URL)).value.get(),
                    "Uniqueness(id)": ctx.metric(A.Uniqueness(["id"])).value.get()}
        b_alg = 0
        for b in table.batches:
            for c in b.values():
                b_alg += c.nbytes()
        kernel = "whole suite (fused scan + 20 group-bys + 10 quantile sorts + MI joints)"
        desc = ("every analyzer on 20 mixed columns (10 numeric, 10 string incl. containsURL over "
                "URL-bearing text), synthetic, 5% nulls (BASELINE.json configs[4], per-GPU shard, "
                "1 GPU)")
        metric_unit = "rows/s"
    else:
        from deequ_amd import _native as N
        from deequ_amd.analyzers import ApproxCountDistinct, Correlation
        from deequ_amd.runners.engine import get_plan, read_row, scan_into
        suite = [ApproxCountDistinct("id"), Correlation("id", "score")]
        specs = [s for a in suite for s in a.aggregation_functions()]
        plan = get_plan(table.schema, specs)
        state = plan.state(0)
        sh = ctypes.c_void_p(stream.cuda_stream)

        def step():
            N.check(N.lib.dq_state_reset(state))
            scan_into(table, plan, state, sh)
            N.check(N.lib.dq_state_sync(state))
            return read_row(plan, state)
        b_alg = 0
        for b in table.batches:
            m = b["id"].length
            b_alg += 2 * nb(m) + 16 * m
        kernel = "dq::scan_kernel<BC_CORR> (co-moments) + dq::scan_kernel<BC_HLL> + finalize"
        desc = ("ApproxCountDistinct(id) + Correlation(id, score) over a synthetic Item table "
                "with fp64 score, 5% nulls (BASELINE.json configs[3], per-GPU shard of 1e10 "
                "rows over 8 GPUs = 1.25e9 rows, 1 GPU)")
        metric_unit = "rows/s"

    for _ in range(warmup):
        res = step()
    if pyprof:
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        step()
        torch.cuda.synchronize(dev)
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(40)
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(40)
        print(buf.getvalue(), file=sys.stderr)
    import gc
    gc_log = []  # (generation, seconds) of every collection, and the host time of each step
    gc_t = {}

    def on_gc(phase, info):
        if phase == "start":
            gc_t["t"] = time.perf_counter()
        else:
            gc_log.append((info["generation"], time.perf_counter() - gc_t.get("t", time.perf_counter()),
                           info.get("collected", 0)))
    gc.callbacks.append(on_gc)
    step_host = []
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        e0[i].record(stream)
        n_gc = len(gc_log)
        ts = time.perf_counter()
        res = step()
        step_host.append((time.perf_counter() - ts, gc_log[n_gc:], torch.cuda.mem_get_info(dev)[0]))
        e1[i].record(stream)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    gc.callbacks.remove(on_gc)
    per_step = [a.elapsed_time(b) for a, b in zip(e0, e1)]
    if verbose:
        print("device ms per step: " + " ".join(f"{x:.1f}" for x in per_step), file=sys.stderr)
    for i, (h, gcs, free) in enumerate(step_host if verbose else []):
        print(f"step {i}: host {h * 1e3:.1f} ms, free {free / 2**30:.1f} GiB, {len(gcs)} gc collections, "
              f"{sum(d for _, d, _ in gcs) * 1e3:.1f} ms, gen2: " +
              ", ".join(f"{d * 1e3:.1f} ms" for g, d, _ in gcs if g == 2), file=sys.stderr)
    dev_ms = sum(per_step) / steps
    achieved = b_alg / (dev_ms * 1e-3)
    cpu = cpu_baseline(workload, cpu_rows, table) if cpu_rows else None
    out = {
        "cpu_baseline": cpu,
        "workload": workload, "desc": desc, "rows": rows, "unit": metric_unit,
        "value": rows / el, "ms_per_step": el * 1e3, "device_ms_per_step": dev_ms,
        "steps": steps, "warmup": warmup, "algorithmic_bytes": b_alg, "frac": achieved / PEAK,
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK / 1e9,
                     "unit": "GB/s", "frac": achieved / PEAK, "algorithmic_bytes": b_alg,
                     "kernel": kernel},
        "result": repr(res)[:300],
    }
    if not verbose:
        del out["result"]
    del table
    return out


def gather_rank_stats(seconds: float, sent: int, recv: int, device: str):
    """Every rank's (seconds, collective bytes sent, received), on every rank: one all-gather of
    three values per rank (on the device over RCCL, host tensors over gloo)."""
    import torch
    import torch.distributed as dist
    from deequ_amd.distributed import _comm_device
    dev = _comm_device(device)
    t = torch.tensor([float(seconds), float(sent), float(recv)], dtype=torch.float64, device=dev)
    out = torch.empty(dist.get_world_size() * 3, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, t)
    v = out.cpu().numpy().reshape(-1, 3)
    return v[:, 0].tolist(), [int(x) for x in v[:, 1]], [int(x) for x in v[:, 2]]


def dist_report(workload: str, per_rank_s, steps: int, rows_per_rank: int, sent, recv,
                backend: str) -> dict:
    """The JSON line of an N-rank run: whole-job rows/s over the slowest rank's time (max over
    ranks), each rank's time per step, and each rank's collective bytes per step (over RCCL the
    xGMI traffic to / from the other ranks)."""
    world = len(per_rank_s)
    t = max(per_rank_s)
    return {"workload": workload, "n_gpus": world, "scaling": "weak", "rows_per_gpu": rows_per_rank,
            "rows": rows_per_rank * world, "unit": "rows/s", "steps": steps,
            "value": rows_per_rank * world * steps / t, "ms_per_step": t / steps * 1e3,
            "per_rank_ms_per_step": [s / steps * 1e3 for s in per_rank_s],
            "collective_bytes_per_step": {"sent": [b / steps for b in sent],
                                          "recv": [b / steps for b in recv], "backend": backend}}


def run_distributed(args, world: int, rank: int, local: int):
    """configs[2] / [3] / [4] on `world` ranks, one per GPU: each rank generates its shard (rows
    [rank * R, (rank + 1) * R) of the same synthetic table, R = --rows) and runs the workload
    through the product's distributed paths -- the scan's state all-gather + rank-ordered merge
    (run_scan_distributed), the groupings' raw-key or partial-aggregate all-to-all
    (compute_frequencies_distributed, via AnalysisRunner) -- K timed steps bracketed by a barrier
    and a device sync on both sides; rank 0 prints one JSON line (dist_report)."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.share_gpu:  # (RCCL takes one rank per device: the rehearsal meets over gloo)
        local = 0
    torch.cuda.set_device(local)
    dist.init_process_group("gloo" if args.share_gpu else "nccl", rank=rank, world_size=world)
    dev = f"cuda:{local}"
    from deequ_amd import distributed as D
    from deequ_amd.runners import AnalysisRunner
    rows = args.rows or {"c3": 1_000_000_000, "c4": 1_250_000_000, "c5": 125_000_000}[args.workload]
    if args.workload == "c5":
        from deequ_amd.synth import profiling_table_device
        table = profiling_table_device(rows, batch_rows=min(args.batch_rows, 1 << 25), device=dev,
                                       start=rank * rows)
        torch.cuda.empty_cache()
        suite = c5_suite()
    else:
        from deequ_amd.synth import item_table_device
        table = item_table_device(rows, seed=9, batch_rows=args.batch_rows, device=dev,
                                  extra=args.workload == "c4", start=rank * rows)
    if args.workload == "c3":
        from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
        suite = [a for c in ("id", "priority")
                 for a in (Uniqueness([c]), Distinctness([c]), Entropy(c), Histogram(c))]
    if args.workload == "c4":
        from deequ_amd.analyzers import ApproxCountDistinct, Correlation
        suite = [ApproxCountDistinct("id"), Correlation("id", "score")]
        specs = [s for a in suite for s in a.aggregation_functions()]

        def step():
            return D.run_scan_distributed(table, specs)
    else:
        def step():
            ctx = AnalysisRunner.do_analysis_run(table, suite)
            bad = [str(a) for a in suite if not ctx.metric(a).value.is_success]
            if bad:
                raise RuntimeError(f"failed metrics: {bad[:3]}")
            return len(suite)
    for _ in range(args.warmup):
        step()
    D.reset_comm_bytes()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    el = time.perf_counter() - t0
    secs, sent, recv = gather_rank_stats(el, D.COMM_BYTES["sent"], D.COMM_BYTES["recv"], dev)
    if rank == 0:
        out = dist_report(args.workload, secs, args.steps, rows, sent, recv, dist.get_backend())
        out["desc"] = (f"BASELINE.json configs[{ {'c3': 2, 'c4': 3, 'c5': 4}[args.workload] }] on "
                       f"{world} GPUs, {rows} synthetic rows per GPU (weak scaling)")
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


def c5_suite():
    from deequ_amd import analyzers as A
    num = ["id"] + [f"numViews_{k}" for k in range(5)] + [f"score_{k}" for k in range(4)]
    strs = ([f"name_{k}" for k in range(3)] + [f"priority_{k}" for k in range(3)]
            + [f"description_{k}" for k in range(4)])
    suite = [A.Size()]
    for c in num + strs:
        suite += [A.Completeness(c), A.ApproxCountDistinct(c), A.Uniqueness([c]),
                  A.Distinctness([c]), A.UniqueValueRatio([c]), A.CountDistinct([c]),
                  A.Entropy(c), A.Histogram(c)]
    for c in num:
        suite += [A.Sum(c), A.Mean(c), A.StandardDeviation(c), A.Minimum(c), A.Maximum(c),
                  A.Compliance(f"{c} non-negative", f"{c} >= 0"), A.ApproxQuantile(c, 0.5)]
    for c in strs:
        suite += [A.DataType(c), A.PatternMatch(c, A.Patterns.URL)]
    suite += [A.Correlation("numViews_0", "score_0"), A.Correlation("numViews_1", "score_1"),
              A.Correlation("id", "numViews_2"),
              A.MutualInformation("priority_0", "priority_1"),
              A.MutualInformation("name_0", "priority_2")]
    return suite


def _host_column(col, n):
    """The first n rows of a device column as host numpy buffers (values, data, validity)."""
    import numpy as np
    vb = (n + 7) // 8
    valid = (col.validity[:vb].cpu().numpy().copy() if col.validity is not None
             else np.full(vb, 0xFF, np.uint8))
    if col.data is not None:  # utf8
        off = col.values[: n + 1].cpu().numpy().astype(np.int32)
        data = col.data[: int(off[-1])].cpu().numpy().copy()
        return off, data if len(data) else np.zeros(1, np.uint8), valid
    return col.values[:n].cpu().numpy().copy(), None, valid


def cpu_baseline(workload: str, cpu_rows: int, table, min_seconds: float = 10.0):
    """The same workload's semantics restated in C/OpenMP (oracle/oracle.c: or_freq = the hash
    Exchange + HashAggregate of Spark local[T], or_hll / or_corr = the partial + final
    aggregation) on a bounded sample: the first rows of the table's first batch, repeated until
    `min_seconds` of CPU work.  kind "port": a CPU restatement of Spark 2.2 deequ -- not Spark."""
    sys.path.insert(0, ROOT)
    from bench import available_cpus
    from oracle import c_oracle as C
    threads, host = available_cpus()
    b0 = table.batches[0]
    first = next(iter(b0.values()))
    n = min(cpu_rows, first.length)
    if workload == "c3":
        cols = {c: _host_column(b0[c], n) for c in ("id", "priority")}

        def one():
            for c, kind in (("id", "long"), ("priority", "string")):
                v, d, m = cols[c]
                C.freq(kind, v, d, m, n, n, null_as_group=True, k=1000, threads=threads)
        what = ("Uniqueness/Distinctness/Entropy + Histogram top-1000 of id and priority: "
                "or_freq (hash-partitioned count, 256 shuffle partitions)")
    elif workload == "c4":
        import numpy as np
        idv, _, idm = _host_column(b0["id"], n)
        sv, _, sm = _host_column(b0["score"], n)
        sv = sv.view(np.float64)

        def one():
            C.hll(5, idv, None, idm, n, threads)
            C.corr(idv, idm, sv, sm, threads)
        what = "ApproxCountDistinct(id) + Correlation(id, score): or_hll + or_corr"
    else:  # c5
        import numpy as np
        from deequ_amd.analyzers import Patterns
        from deequ_amd.regex import compile_java_regex
        url = compile_java_regex(Patterns.URL)
        names = [f.name for f in table.schema.fields]
        cols = {c: _host_column(b0[c], n) for c in names}
        ints = [c for c in names if c == "id" or c.startswith("numViews")]
        dbls = [c for c in names if c.startswith("score")]
        strs = [c for c in names if c not in ints and c not in dbls]
        nv2 = cols["numViews_2"][0].astype(np.float64)  # (Correlation(id, numViews_2) in doubles)

        def one():
            for c in ints:
                v, _, m = cols[c]
                C.numeric_i64(v, m, 17, 0, threads)          # Size..Max, Compliance(>= 0)
                C.hll(5, v, None, m, n, threads)
                C.freq("long", v, None, m, n, n, True, 1000, threads)
                np.sort(v)                                   # ApproxQuantile (sort stand-in)
            for c in dbls:
                v, _, m = cols[c]
                d = v.view(np.float64)
                C.numeric_f64(d, m, 0.0, threads)
                C.hll(7, d, None, m, n, threads)
                C.freq("long", v, None, m, n, n, True, 1000, threads)  # on the value bits
                np.sort(d)
            for c in strs:
                o, d, m = cols[c]
                C.hll(8, o, d, m, n, threads)
                C.freq("string", o, d, m, n, n, True, 1000, threads)
                C.dfa_count(o, d, m, n, url, threads)
                C.dtype_utf8(o, d, m, n, threads)            # DataType
            for x, y in (("numViews_0", "score_0"), ("numViews_1", "score_1")):
                C.corr(cols[x][0], cols[x][2], cols[y][0].view(np.float64), cols[y][2], threads)
            C.corr(cols["id"][0], cols["id"][2], nv2, cols["numViews_2"][2], threads)
            for x, y in (("priority_0", "priority_1"), ("name_0", "priority_2")):
                C.mi_utf8(cols[x], cols[y], n, n, threads)   # MutualInformation
        what = ("the whole configs[4] suite: per numeric column the scan aggregates "
                "(or_numeric_i64/_f64), or_hll, or_freq (Uniqueness..Histogram) and a numpy sort "
                "for ApproxQuantile; per string column or_hll, or_freq, the URL PatternMatch as a "
                "DFA walk (or_dfa_count) and DataType (or_dtype_utf8); three Correlations; the two "
                "MutualInformations (or_mi_utf8: joint hash aggregation + marginals)")
    one()
    reps, t0 = 0, time.perf_counter()
    while True:
        one()
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds or reps >= 1000:
            break
    return {"value": reps * n / el, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"{what} over the first {n} rows of the same synthetic table x {reps} passes "
                      f"({el:.1f} s), oracle/oracle.c, OpenMP, {threads} threads = Spark "
                      f"local[{threads}] (every CPU this process may use; the host has {host}) "
                      f"-- a CPU restatement of Spark 2.2 deequ semantics, not Spark"}


if __name__ == "__main__":
    main()
