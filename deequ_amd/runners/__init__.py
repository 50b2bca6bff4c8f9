"""AnalysisRunner (reference: analyzers/runners/AnalysisRunner.scala, AnalyzerContext.scala,
AnalysisRunBuilder.scala, analyzers/Analysis.scala).

The planning logic is the reference's, line by line in behaviour: repository reuse, precondition
failures, the scan-shareable / grouping partition, ONE fused scan for every shareable analyzer
(here: one engine launch instead of one Spark job), one frequency table per sorted grouping-column
set with one shared aggregation over it, and failure isolation (a failing shared scan fails every
shareable analyzer, a failing ``from_aggregation_result`` fails only its analyzer).
"""
from __future__ import annotations

import dataclasses
import functools
import gc
import threading
import json
import os
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from .. import _native as N
from ..analyzers.base import (Analyzer, GroupingAnalyzer, Preconditions, ScanShareableAnalyzer)
from ..analyzers.scan import ApproxCountDistinct
from ..analyzers.grouping import (FrequenciesAndNumRows, Histogram, KeyedFrequencies,
                                  ScanShareableFrequencyBasedAnalyzer, compute_frequencies,
                                  frequency_row)
from ..exceptions import ReusingNotPossibleResultsMissingException
from ..metrics import DoubleMetric
from ..distributed import compute_frequencies_distributed, is_distributed, run_scan_distributed
from .engine import run_scan


@dataclass
class AnalyzerContext:
    """AnalyzerContext.scala:29-42"""
    metric_map: Dict[Analyzer, object] = field(default_factory=dict)

    @staticmethod
    def empty() -> "AnalyzerContext":
        return AnalyzerContext({})

    def all_metrics(self) -> list:
        return list(self.metric_map.values())

    def __add__(self, other: "AnalyzerContext") -> "AnalyzerContext":
        merged = dict(self.metric_map)
        merged.update(other.metric_map)  # right side wins, like Map ++ Map
        return AnalyzerContext(merged)

    def metric(self, analyzer: Analyzer):
        return self.metric_map.get(analyzer)

    @staticmethod
    def success_metrics_as_rows(ctx: "AnalyzerContext", for_analyzers: Sequence = ()) -> list:
        rows = []
        for a, m in ctx.metric_map.items():
            if for_analyzers and a not in for_analyzers:
                continue
            if not m.value.is_success:
                continue
            for d in m.flatten():
                rows.append({"entity": str(d.entity), "instance": d.instance, "name": d.name,
                             "value": d.value.get()})
        return rows

    @staticmethod
    def success_metrics_as_json(ctx: "AnalyzerContext", for_analyzers: Sequence = ()) -> str:
        return json.dumps(AnalyzerContext.success_metrics_as_rows(ctx, for_analyzers))


# Runs may overlap (threads): only the outermost one pauses the cyclic GC and restores its
# previous state, so an inner run ending never re-enables collection under an outer one.
_gc_lock = threading.Lock()
_gc_depth = 0
_gc_was_enabled = False


def _gc_pause_enter():
    global _gc_depth, _gc_was_enabled
    with _gc_lock:
        if _gc_depth == 0:
            _gc_was_enabled = gc.isenabled()
            gc.disable()
        _gc_depth += 1


def _gc_pause_exit():
    global _gc_depth
    with _gc_lock:
        _gc_depth -= 1
        if _gc_depth == 0 and _gc_was_enabled:
            gc.enable()


@dataclass
class AnalysisRunnerRepositoryOptions:
    metrics_repository: object = None
    reuse_existing_results_for_key: object = None
    fail_if_results_for_reusing_missing: bool = False
    save_or_append_results_with_key: object = None


class AnalysisRunner:
    """AnalysisRunner.scala"""

    @staticmethod
    def on_data(data) -> "AnalysisRunBuilder":
        return AnalysisRunBuilder(data)

    @staticmethod
    def run(data, analysis: "Analysis", aggregate_with=None, save_states_with=None) -> AnalyzerContext:
        return AnalysisRunner.do_analysis_run(data, analysis.analyzers, aggregate_with,
                                              save_states_with)

    @staticmethod
    def do_analysis_run(data, analyzers: Sequence[Analyzer], aggregate_with=None,
                        save_states_with=None,
                        repository_options: Optional[AnalysisRunnerRepositoryOptions] = None
                        ) -> AnalyzerContext:
        """AnalysisRunner.doAnalysisRun (AnalysisRunner.scala:98-193).  Python's cyclic garbage
        collector is paused for the run: a full (generation-2) collection walks every object of
        the process -- 45-78 ms with torch loaded, in about every other configs[4] step -- while
        a run leaves only a few dozen cycles, which the next collection after it frees."""
        if not analyzers:
            return AnalyzerContext.empty()
        _gc_pause_enter()
        try:
            return AnalysisRunner._do_analysis_run(data, analyzers, aggregate_with,
                                                   save_states_with, repository_options)
        finally:
            _gc_pause_exit()

    @staticmethod
    def _do_analysis_run(data, analyzers, aggregate_with, save_states_with, repository_options):
        opts = repository_options or AnalysisRunnerRepositoryOptions()
        previous = AnalyzerContext.empty()
        if opts.metrics_repository is not None and opts.reuse_existing_results_for_key is not None:
            previous = opts.metrics_repository.load_by_key(
                opts.reuse_existing_results_for_key) or AnalyzerContext.empty()
        already = set(previous.metric_map.keys())
        # dedupe preserving order (case classes: equal analyzers run once); by hash, not by list
        # scans (O(n^2) dataclass comparisons were ~20 ms of host time per configs[4] run)
        to_run: List[Analyzer] = []
        try:
            seen = set(already)
            for a in analyzers:
                if a not in seen:
                    seen.add(a)
                    to_run.append(a)
        except TypeError:  # an analyzer that does not hash: compare by equality
            to_run = []
            for a in analyzers:
                if a not in already and a not in to_run:
                    to_run.append(a)
        if opts.fail_if_results_for_reusing_missing and to_run:
            raise ReusingNotPossibleResultsMissingException(
                "Could not find all necessary results in the MetricsRepository, the calculation of "
                f"the metrics for these analyzers would be needed: {', '.join(map(str, to_run))}")
        schema = data.schema
        passed, failed = [], []
        for a in to_run:
            ok = Preconditions.find_first_failing(schema, a.preconditions()) is None
            (passed if ok else failed).append(a)
        precondition_failures = _precondition_failure_metrics(failed, schema)
        grouping = [a for a in passed if isinstance(a, GroupingAnalyzer)]
        scanning = [a for a in passed if not isinstance(a, GroupingAnalyzer)]
        groups: Dict[tuple, List[Analyzer]] = {}
        for a in grouping:
            groups.setdefault(tuple(sorted(a.grouping_columns())), []).append(a)
        # Every grouping (one frequency table per column set), the shared scan and each other
        # scanning analyzer are independent jobs, run one at a time by default (_job_workers;
        # DQ_RUN_WORKERS > 1 runs them on that many HIP streams at once); the metrics are
        # assembled in the reference's order.
        hist_cols = _histogram_columns_for_groupings(data, grouping, scanning, aggregate_with,
                                                     save_states_with)
        hist_jobs = []
        for col in hist_cols:
            hists = [h for h in scanning if isinstance(h, Histogram) and h.column == col]
            hist_jobs.append(functools.partial(_histogram_and_grouping_job, data, col, hists,
                                               groups.pop((col,)), aggregate_with,
                                               save_states_with))
        hist_set = set(hist_cols)
        scanning = [a for a in scanning if not (isinstance(a, Histogram) and a.column in hist_set)]
        shareable = [a for a in scanning if isinstance(a, ScanShareableAnalyzer)]
        others = [a for a in scanning if not isinstance(a, ScanShareableAnalyzer)]
        # ApproxCountDistinct(c) beside a Histogram(c) table built in this run: the registers come
        # from the table's groups when it has few of them (_hll_from_tables), so the scan skips c
        hll_cols = _hll_table_columns(shareable, hist_cols, aggregate_with, save_states_with, data)
        hll_words: Dict[str, tuple] = {}
        for job in hist_jobs:
            if job.args[1] in hll_cols:
                job.keywords["hll_words"] = hll_words
        scan_jobs = [functools.partial(_run_scanning_analyzers, data, shareable, aggregate_with,
                                       save_states_with, hll_words=hll_words if hll_cols else None)] + \
            [functools.partial(_run_scanning_analyzers, data, [a], aggregate_with, save_states_with)
             for a in others]
        group_jobs = [functools.partial(_run_grouping_analyzers, data, list(cols), group,
                                        aggregate_with, save_states_with, None, None)
                      for cols, group in groups.items()]
        # multi-column groupings (MutualInformation, Uniqueness over column sets) are the
        # longest jobs: they start first
        jobs = group_jobs + hist_jobs + scan_jobs
        order = sorted(range(len(jobs)), key=lambda j: -_job_weight(jobs[j]))
        workers = _job_workers(data, [list(c) for c in groups] + [[c] for c in hist_cols],
                               aggregate_with, save_states_with)
        done = _run_jobs(data, [jobs[j] for j in order], workers)
        out = [None] * len(jobs)
        for j, r in zip(order, done):
            out[j] = r
        group_out = out[:len(group_jobs)]
        hist_out = out[len(group_jobs):len(group_jobs) + len(hist_jobs)]
        scan_out = out[len(group_jobs) + len(hist_jobs):]
        non_grouped = AnalyzerContext.empty()
        for ctx in scan_out:
            non_grouped = non_grouped + ctx
        grouped = AnalyzerContext.empty()
        for hist_ctx, _ in hist_out:
            non_grouped = non_grouped + hist_ctx
        for _, grouping_ctx in hist_out:
            grouped = grouped + grouping_ctx
        for _, metrics in group_out:
            grouped = grouped + metrics
        result = previous + precondition_failures + non_grouped + grouped
        if opts.metrics_repository is not None and opts.save_or_append_results_with_key is not None:
            current = opts.metrics_repository.load_by_key(opts.save_or_append_results_with_key) \
                or AnalyzerContext.empty()
            opts.metrics_repository.save(opts.save_or_append_results_with_key, current + result)
        return result

    @staticmethod
    def run_on_aggregated_states(schema, analysis: "Analysis", state_loaders: Sequence,
                                 save_states_with=None) -> AnalyzerContext:
        """AnalysisRunner.runOnAggregatedStates (AnalysisRunner.scala:375-446): metrics from
        persisted partition states, no data touched."""
        from ..analyzers.state_provider import InMemoryStateProvider
        if not analysis.analyzers or not state_loaders:
            return AnalyzerContext.empty()
        analyzers = list(analysis.analyzers)
        passed = [a for a in analyzers if Preconditions.find_first_failing(schema, a.preconditions()) is None]
        failed = [a for a in analyzers if a not in passed]
        precondition_failures = _precondition_failure_metrics(failed, schema)
        aggregated = InMemoryStateProvider()
        for a in passed:
            for loader in state_loaders:
                a.aggregate_state_to(aggregated, loader, aggregated)
        grouping = [a for a in passed if isinstance(a, GroupingAnalyzer)]
        scanning = [a for a in passed if a not in grouping]
        non_grouped = {}
        for a in scanning:
            m = a.load_state_and_compute_metric(aggregated)
            if m is not None:
                non_grouped[a] = m
        grouped = AnalyzerContext.empty()
        groups: Dict[tuple, List[Analyzer]] = {}
        for a in grouping:
            groups.setdefault(tuple(sorted(a.grouping_columns())), []).append(a)
        for _, group in groups.items():
            states = [aggregated.load(a) for a in group]
            states = [s for s in states if s is not None]
            if not states:
                raise AssertionError("requirement failed")
            grouped = grouped + _run_analyzers_for_particular_grouping(states[0], group,
                                                                        save_states_with)
        return precondition_failures + AnalyzerContext(non_grouped) + grouped


def _histogram_and_grouping_job(data, col, hists, group, aggregate_with, save_states_with,
                                hll_words=None):
    """Histogram(col) and the grouping of [col] from one table (_histogram_columns_for_groupings).
    Returns (Histogram metrics, grouping metrics).  If the Histogram table cannot be built, both
    run (and fail) on their own, as in the reference's two group-bys.  hll_words (a dict): the
    column's HLL registers from the table's groups are put there (_hll_from_tables)."""
    st = _histogram_and_grouping_launch(data, col, hists, group, aggregate_with, save_states_with,
                                        hll_words)
    _histogram_and_grouping_device(st)
    return _histogram_and_grouping_host(st)


# A column's ApproxCountDistinct is taken from its Histogram table (not scanned) when phase A
# collapsed the column's repeated keys to at most this many partitioned records per row: the
# records are hashed on the device (dq_freq_hll) instead of the rows.  Measured on configs[4]
# (DESIGN.md §4.1): a table with a record per row (id, score) took 1.6 ms to hash its 125 M
# records, while the fused scan, bound by its string columns, ran no faster without the column.
kHllTableRecordsPerRow = 1.0 / 64


def _hll_table_columns(shareable, hist_cols, aggregate_with, save_states_with, data) -> set:
    """Columns whose ApproxCountDistinct (no where) may come from this run's Histogram table of
    the column (DQ_HLL_FROM_TABLE=0 turns it off): one process, no state I/O (a loaded or saved
    HLL state keeps its scan), and the jobs run one at a time (the scan job runs after the
    Histogram jobs that fill the registers)."""
    if (aggregate_with is not None or save_states_with is not None or is_distributed(data)
            or os.environ.get("DQ_HLL_FROM_TABLE", "1") == "0"
            or int(os.environ.get("DQ_RUN_WORKERS", "1") or 1) > 1):
        return set()
    want = {a.column for a in shareable if isinstance(a, ApproxCountDistinct) and a.where is None}
    return want & set(hist_cols)


def _hll_from_table(st, hll_words) -> None:
    """The Histogram table's HLL registers into hll_words[col] when it has few records."""
    hs, col = st[6], st[1]
    if hs is None or hll_words is None:
        return
    per_row = float(os.environ.get("DQ_HLL_TABLE_RECORDS_PER_ROW", kHllTableRecordsPerRow))
    cap = int(max(1, int(hs.num_rows)) * per_row)
    try:
        words = hs.frequencies.hll_words(cap)
    except Exception:  # noqa: BLE001  (the scan computes it instead)
        words = None
    if words is not None:
        hll_words[col] = words


# The job in three stages, so that the sequential runner (_run_jobs) can run one job's host-only
# stage while the device runs the next job's phase A: launch (the table's batches queued),
# device (every device result the metrics need: finalize, the top-k, the NULL-group counts --
# afterwards the table's calls answer from its caches), host (decoding and metric objects).
def _histogram_and_grouping_launch(data, col, hists, group, aggregate_with, save_states_with,
                                   hll_words=None):
    try:
        hs = hists[0].compute_state_from(data)
    except Exception:  # noqa: BLE001
        hs = None
    return (data, col, hists, group, aggregate_with, save_states_with, hs, hll_words)


def _histogram_and_grouping_device(st):
    hs, hists = st[6], st[2]
    if hs is None:
        return
    _hll_from_table(st, st[7])
    try:
        if hs.binning_udf is None and hists and all(h.binning_udf is None for h in hists):
            ft = hs.frequencies
            if os.environ.get("DQ_RUN_TRACE") == "3":  # (the calls' host times)
                t = [time.perf_counter()]
                ft.topk_raw(max(h.max_detail_bins for h in hists) + 2)
                t.append(time.perf_counter())
                ft.null_literal()
                t.append(time.perf_counter())
                ft.count()
                t.append(time.perf_counter())
                print("[dq run] device calls us: " + " ".join(
                    f"{1e6 * (b - a):.1f}" for a, b in zip(t, t[1:])), file=sys.stderr)
                return
            ft.topk_raw(max(h.max_detail_bins for h in hists) + 2)
            ft.null_literal()
            ft.count()
    except Exception:  # noqa: BLE001  (the host stage meets the error again and records it)
        pass


def _histogram_and_grouping_host(st):
    data, col, hists, group, aggregate_with, save_states_with, hs, _ = st
    if hs is None:
        return (_run_scanning_analyzers(data, hists, aggregate_with, save_states_with),
                _run_grouping_analyzers(data, [col], group, aggregate_with, save_states_with,
                                        None, None)[1])
    hist_metrics = {}
    for h in hists:
        hist_metrics[h] = h.compute_metric_from(dataclasses.replace(hs, binning_udf=h.binning_udf))
    state = FrequenciesAndNumRows(KeyedFrequencies(hs.frequencies), hs.num_rows)
    if data.schema[col].dtype in (N.FLOAT32, N.FLOAT64) and hs.frequencies.folded_nan_rows() != 0:
        state = None  # (NaN payloads folded for Histogram: the grouping groups the column itself)
    _, metrics = _run_grouping_analyzers(data, [col], group, aggregate_with, save_states_with,
                                         None, state)
    return AnalyzerContext(hist_metrics), metrics


def _job_name(job) -> str:
    if job.func is _run_scanning_analyzers:
        return "scan " + ",".join(type(a).__name__ for a in job.args[1])
    return f"{job.func.__name__} {job.args[1]}"


def _job_weight(job) -> int:
    """Submission order of the jobs: groupings over several columns first, then one-column
    groupings and Histograms, then the scans (ties keep their order)."""
    if job.func is _run_grouping_analyzers:
        return 2 if len(job.args[1]) > 1 else 1
    return 1 if job.func is _histogram_and_grouping_job else 0


def _job_workers(data, key_sets, aggregate_with, save_states_with) -> int:
    """How many jobs run at once: DQ_RUN_WORKERS (default 1), one for a row-sharded table (every
    rank must issue its collectives in the same order) or when states are loaded or persisted,
    and no more than the free device memory holds of the largest group-by's buffers (about 64
    bytes per row plus twice its key bytes).  Measured on configs[4]: four
    concurrent jobs took 2.5-4.0 s per step against 0.42 s for one at a time, so concurrency is
    opt-in."""
    if is_distributed(data) or aggregate_with is not None or save_states_with is not None:
        return 1
    try:
        workers = int(os.environ.get("DQ_RUN_WORKERS", "1"))
    except ValueError:
        workers = 1
    if workers <= 1:
        return 1
    import torch
    if not torch.cuda.is_available():
        return 1
    rows = data.num_rows
    per_job = 0
    for cols in key_sets:
        key_bytes = sum(b[c].nbytes() for b in data.batches for c in cols if c in b)
        per_job = max(per_job, 64 * rows + 2 * key_bytes)
    if per_job:
        free, _ = torch.cuda.mem_get_info(data.device_index())
        workers = min(workers, max(1, int(0.8 * free) // per_job))
    return workers


def _histogram_scan_launch(data, analyzers, aggregate_with, save_states_with):
    """A scanning job of one Histogram (a column whose table does not serve its grouping) in the
    three stages of _histogram_and_grouping_job: Analyzer.calculate, split."""
    a = analyzers[0]
    try:
        for condition in a.preconditions():
            condition(data.schema)
        return (a, a.compute_state_from(data), None)
    except Exception as e:  # noqa: BLE001
        return (a, None, e)


def _histogram_scan_device(st):
    a, state, err = st
    if err is not None or state is None or state.binning_udf is not None:
        return
    try:
        state.frequencies.topk_raw(a.max_detail_bins + 2)
        state.frequencies.null_literal()
        state.frequencies.count()
    except Exception:  # noqa: BLE001  (the host stage meets the error again and records it)
        pass


def _histogram_scan_host(st):
    a, state, err = st
    if err is None:
        try:
            return AnalyzerContext({a: a.calculate_metric(state, None, None)})
        except Exception as e:  # noqa: BLE001
            err = e
    return AnalyzerContext({a: a.to_failure_metric(err)})


def _stages_of(job):
    """(launch, device, host) of a job the sequential runner may overlap, else None."""
    if job.func is _histogram_and_grouping_job:
        return (_histogram_and_grouping_launch, _histogram_and_grouping_device,
                _histogram_and_grouping_host)
    if (job.func is _run_scanning_analyzers and len(job.args[1]) == 1
            and isinstance(job.args[1][0], Histogram) and job.args[2] is None
            and job.args[3] is None):
        return _histogram_scan_launch, _histogram_scan_device, _histogram_scan_host
    return None


def _launch_failed(st) -> bool:
    """The launch stage of _histogram_and_grouping_job / _histogram_scan_launch built no table."""
    return st[6] is None if len(st) == 8 else st[2] is not None


def _table_fits_beside(job) -> bool:
    """Whether job's group-by table fits on the device while the previous job's table is still
    held: its estimate (about 64 bytes per row plus twice its key bytes, as _job_workers) against
    the device's free bytes plus the idle blocks of the engine's cache."""
    data = job.args[0]
    cols = [job.args[1]] if job.func is _histogram_and_grouping_job else [job.args[1][0].column]
    try:
        import torch
        dev = data.device_index()
        need = 64 * data.num_rows + 2 * sum(b[c].nbytes() for b in data.batches for c in cols
                                            if c in b)
        free, _ = torch.cuda.mem_get_info(dev)
        from .. import _native as N
        return free + int(N.lib.dq_cached_device_bytes(dev)) >= need
    except Exception:  # noqa: BLE001  (no estimate: do not overlap)
        return False


def _run_jobs_pipelined(jobs, trace: bool = False) -> list:
    """One job at a time, except that a Histogram job's host-only stage runs after the next
    Histogram job's batches are queued, so the device works through that job's phase A
    meanwhile (the host stage touches only the finished table's caches).  That holds two tables
    on the device at once, so it is done only when the next table's estimate fits beside the
    held one (_table_fits_beside); a launch that fails beside it runs again after the held
    table's host stage.  trace (DQ_RUN_TRACE=2): each stage's wall time on stderr."""
    out = [None] * len(jobs)
    pending = None  # (index, host stage, state) of a job whose host stage has not run
    clock = time.perf_counter

    def stage(what, i, fn, *a, **kw):
        if not trace:
            return fn(*a, **kw)
        t0 = clock()
        r = fn(*a, **kw)
        print(f"[dq run] {1e3 * t0:12.3f} {1e6 * (clock() - t0):9.1f} us {what} "
              f"{_job_name(jobs[i])}", file=sys.stderr)
        return r

    for i, job in enumerate(jobs):
        stages = _stages_of(job)
        if stages is not None:
            launch, device, host = stages
            if pending is not None and not _table_fits_beside(job):
                out[pending[0]] = stage("host", pending[0], pending[1], pending[2])
                pending = None
            st = stage("launch", i, launch, *job.args, **job.keywords)
            if pending is not None:
                out[pending[0]] = stage("host", pending[0], pending[1], pending[2])
                pending = None
                if _launch_failed(st):  # (maybe out of memory beside the other table: again alone)
                    st = stage("launch", i, launch, *job.args, **job.keywords)
            stage("device", i, device, st)
            pending = (i, host, st)
            continue
        if pending is not None:
            out[pending[0]] = stage("host", pending[0], pending[1], pending[2])
            pending = None
        out[i] = stage("job", i, job)
    if pending is not None:
        out[pending[0]] = stage("host", pending[0], pending[1], pending[2])
    return out


def _run_jobs(data, jobs, workers: int) -> list:
    """Runs the jobs, `workers` at a time, each on a HIP stream of its own (a thread per job: the
    engine's calls release the GIL), and returns their results in order.  Each stream first waits
    for the caller's stream (the table's buffers), and the caller's stream waits for all of them
    at the end."""
    if workers <= 1 or len(jobs) <= 1:
        trace = os.environ.get("DQ_RUN_TRACE", "")
        if trace in ("", "2", "3"):
            if is_distributed(data):  # (every rank keeps the plain order of its collectives)
                return [job() for job in jobs]
            return _run_jobs_pipelined(jobs, trace in ("2", "3"))
        out = []
        for job in jobs:  # DQ_RUN_TRACE=1: each job's wall time on stderr
            t0 = time.perf_counter()
            out.append(job())
            print(f"[dq run] {time.perf_counter() - t0:9.4f} s {_job_name(job)}", file=sys.stderr)
        return out
    import queue
    from concurrent.futures import ThreadPoolExecutor
    import torch
    dev = data.device_index()
    main = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(workers)]
    idle = queue.SimpleQueue()
    for s in streams:
        idle.put(s)

    def run(job):
        s = idle.get()
        try:
            with torch.cuda.device(dev), torch.cuda.stream(s):
                s.wait_stream(main)
                return job()
        finally:
            idle.put(s)

    try:
        with ThreadPoolExecutor(max_workers=workers) as pool:
            futures = [pool.submit(run, job) for job in jobs]
            return [f.result() for f in futures]
    finally:
        for s in streams:
            main.wait_stream(s)


def _precondition_failure_metrics(failed: Sequence[Analyzer], schema) -> AnalyzerContext:
    out = {}
    for a in failed:
        e = Preconditions.find_first_failing(schema, a.preconditions())
        out[a] = a.to_failure_metric(e)
    return AnalyzerContext(out)


def _run_scanning_analyzers(data, analyzers: Sequence[Analyzer], aggregate_with,
                            save_states_with, hll_words=None) -> AnalyzerContext:
    """AnalysisRunner.runScanningAnalyzers (AnalysisRunner.scala:279-326).  hll_words: the
    register words of columns whose Histogram table yielded them (_hll_from_tables): those
    ApproxCountDistincts take their state from there and leave the fused scan."""
    shareable = [a for a in analyzers if isinstance(a, ScanShareableAnalyzer)]
    others = [a for a in analyzers if not isinstance(a, ScanShareableAnalyzer)]
    results: Dict[Analyzer, object] = {}
    if hll_words:
        from ..analyzers.scan import ApproxCountDistinctState
        kept = []
        for a in shareable:
            if isinstance(a, ApproxCountDistinct) and a.where is None and a.column in hll_words:
                results[a] = a.calculate_metric(ApproxCountDistinctState(hll_words[a.column]),
                                                aggregate_with, save_states_with)
            else:
                kept.append(a)
        shareable = kept
    if shareable:
        try:
            aggregations = [spec for a in shareable for spec in a.aggregation_functions()]
            offsets = [0]
            for a in shareable:
                offsets.append(offsets[-1] + len(a.aggregation_functions()))
            # ONE fused pass (the reference's single Spark job); over a row-sharded table, every
            # rank's pass + the all-gather and rank-ordered merge of the states
            row = (run_scan_distributed if is_distributed(data) else run_scan)(data, aggregations)
            for a, off in zip(shareable, offsets):
                try:
                    results[a] = a.metric_from_aggregation_result(row, off, aggregate_with,
                                                                  save_states_with)
                except Exception as e:  # noqa: BLE001
                    results[a] = a.to_failure_metric(e)
        except Exception as e:  # noqa: BLE001
            for a in shareable:
                results[a] = a.to_failure_metric(e)
    for a in others:
        results[a] = a.calculate(data, aggregate_with, save_states_with)
    return AnalyzerContext(results)


def _histogram_columns_for_groupings(data, grouping, scanning, aggregate_with,
                                     save_states_with) -> List[str]:
    """Histogram(c) and the grouping of [c] (Uniqueness, Entropy, ...) are two group-bys of the
    same column in the reference (AnalysisRunner.scala:249-277 and 321-323).  Where the Histogram
    table also yields the grouping exactly (Histogram.table_serves_grouping: the same non-NULL
    groups), the column is grouped once and both read that table.  Not done when states are
    aggregated or persisted, which keep their own tables."""
    if aggregate_with is not None or save_states_with is not None or is_distributed(data):
        return []
    grouped = {tuple(sorted(a.grouping_columns())) for a in grouping}
    out: List[str] = []
    for h in scanning:
        if not isinstance(h, Histogram) or h.column in out or (h.column,) not in grouped:
            continue
        if Histogram.table_serves_grouping(data, h.column):
            out.append(h.column)
    return out


def _run_grouping_analyzers(data, grouping_columns, analyzers, aggregate_with, save_states_with,
                            num_rows_of_data, state=None):
    """AnalysisRunner.runGroupingAnalyzers (AnalysisRunner.scala:249-277).  The reference's
    groupBy is lazy, so a failure of the grouping surfaces inside the one aggregation over the
    frequencies, whose try fails every analyzer of the grouping (:490-505); the engine's eager
    group-by error is mapped the same way."""
    if state is None:
        try:
            if is_distributed(data):  # local partial groupBy + hash repartition by owner rank
                state = compute_frequencies_distributed(data, grouping_columns)
            else:
                state = compute_frequencies(data, grouping_columns)
        except Exception as e:  # noqa: BLE001
            return None, AnalyzerContext({a: a.to_failure_metric(e) for a in analyzers})
    sample = analyzers[0]
    if aggregate_with is not None:
        prev = aggregate_with.load(sample)
        if prev is not None:
            state = state.sum(prev)
    return state.num_rows, _run_analyzers_for_particular_grouping(state, analyzers, save_states_with)


def _run_analyzers_for_particular_grouping(state: FrequenciesAndNumRows, analyzers,
                                           save_states_with) -> AnalyzerContext:
    """AnalysisRunner.runAnalyzersForParticularGrouping (AnalysisRunner.scala:466-534)."""
    num_rows = state.num_rows
    shareable = [a for a in analyzers if isinstance(a, ScanShareableFrequencyBasedAnalyzer)]
    others = [a for a in analyzers if a not in shareable]
    results: Dict[Analyzer, object] = {}
    if shareable:
        try:
            aggs = [g for a in shareable for g in a.aggregation_functions(num_rows)]
            offsets = [0]
            for a in shareable:
                offsets.append(offsets[-1] + len(a.aggregation_functions(num_rows)))
            row = frequency_row(state.frequencies.summarize(), aggs, num_rows)
            for a, off in zip(shareable, offsets):
                try:
                    results[a] = a.from_aggregation_result(row, off)
                except Exception as e:  # noqa: BLE001
                    results[a] = a.to_failure_metric(e)
        except Exception as e:  # noqa: BLE001
            for a in shareable:
                results[a] = a.to_failure_metric(e)
    try:
        for a in others:
            results[a] = a.compute_metric_from(state)
    except Exception as e:  # noqa: BLE001
        for a in others:
            results[a] = a.to_failure_metric(e)
    if save_states_with is not None:
        save_states_with.persist(analyzers[0], state)
    return AnalyzerContext(results)


@dataclass
class Analysis:
    """analyzers/Analysis.scala"""
    analyzers: List[Analyzer] = field(default_factory=list)

    def add_analyzer(self, analyzer: Analyzer) -> "Analysis":
        return Analysis(self.analyzers + [analyzer])

    def add_analyzers(self, analyzers: Sequence[Analyzer]) -> "Analysis":
        return Analysis(self.analyzers + list(analyzers))

    def run(self, data, aggregate_with=None, save_states_with=None) -> AnalyzerContext:
        return AnalysisRunner.do_analysis_run(data, self.analyzers, aggregate_with, save_states_with)


class AnalysisRunBuilder:
    """AnalysisRunBuilder.scala:61-186"""

    def __init__(self, data):
        self.data = data
        self.analyzers: List[Analyzer] = []
        self.repository_options = AnalysisRunnerRepositoryOptions()

    def add_analyzer(self, analyzer: Analyzer) -> "AnalysisRunBuilder":
        self.analyzers.append(analyzer)
        return self

    def add_analyzers(self, analyzers: Sequence[Analyzer]) -> "AnalysisRunBuilder":
        self.analyzers.extend(analyzers)
        return self

    def use_repository(self, repository) -> "AnalysisRunBuilder":
        self.repository_options.metrics_repository = repository
        return self

    def reuse_existing_results_for_key(self, key, fail_if_results_missing: bool = False):
        self.repository_options.reuse_existing_results_for_key = key
        self.repository_options.fail_if_results_for_reusing_missing = fail_if_results_missing
        return self

    def save_or_append_result(self, key) -> "AnalysisRunBuilder":
        self.repository_options.save_or_append_results_with_key = key
        return self

    def run(self) -> AnalyzerContext:
        return AnalysisRunner.do_analysis_run(self.data, self.analyzers,
                                              repository_options=self.repository_options)


__all__ = ["AnalyzerContext", "AnalysisRunner", "AnalysisRunBuilder", "Analysis",
           "AnalysisRunnerRepositoryOptions", "DoubleMetric"]
