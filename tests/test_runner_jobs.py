"""Host logic of AnalysisRunner's job split (runners/__init__.py: _run_jobs, _job_weight,
_job_workers): the order jobs start in, results returned in submission order, and the cases that
must stay on one stream (row-sharded tables, state providers)."""
import functools

from deequ_amd.runners import (_histogram_and_grouping_job, _job_weight, _job_workers, _run_grouping_analyzers,
                               _run_jobs, _run_scanning_analyzers)


class _Table:
    def __init__(self):
        self.batches = []
        self.num_rows = 0

    def device_index(self):
        return 0


def test_results_come_back_in_submission_order():
    calls = []

    def job(i):
        calls.append(i)
        return i * i

    jobs = [functools.partial(job, i) for i in range(5)]
    assert _run_jobs(_Table(), jobs, 1) == [0, 1, 4, 9, 16]
    assert calls == [0, 1, 2, 3, 4]


def test_multi_column_groupings_start_first():
    data = _Table()
    multi = functools.partial(_run_grouping_analyzers, data, ["a", "b"], [], None, None, None, None)
    single = functools.partial(_run_grouping_analyzers, data, ["a"], [], None, None, None, None)
    hist = functools.partial(_histogram_and_grouping_job, data, "a", [], [], None, None)
    scan = functools.partial(_run_scanning_analyzers, data, [], None, None)
    jobs = [scan, single, hist, multi]
    order = sorted(range(len(jobs)), key=lambda j: -_job_weight(jobs[j]))
    assert [jobs[j] for j in order] == [multi, single, hist, scan]


def test_one_worker_when_states_are_loaded_or_saved(monkeypatch):
    monkeypatch.setenv("DQ_RUN_WORKERS", "4")
    data = _Table()
    assert _job_workers(data, [["a"]], object(), None) == 1
    assert _job_workers(data, [["a"]], None, object()) == 1
    monkeypatch.setenv("DQ_RUN_WORKERS", "1")
    assert _job_workers(data, [["a"]], None, None) == 1
    monkeypatch.delenv("DQ_RUN_WORKERS")  # one at a time unless asked
    assert _job_workers(data, [["a"]], None, None) == 1
