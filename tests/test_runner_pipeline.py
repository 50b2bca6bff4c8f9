"""The sequential runner's overlap of staged jobs (runners/__init__.py _run_jobs_pipelined): a
staged job's host stage runs after the next staged job's launch and before that job's device
stage, every result lands in its own job's slot, and a plain job first drains the pending host
stage.  Host only (fake stages)."""
import functools

from deequ_amd import runners as R


def _plain(log, name):
    log.append(("job", name))
    return name


def _staged(name):  # a marker job; its stages come from the patched _stages_of
    raise AssertionError("a staged job is never called whole")


def test_staged_jobs_overlap_host_with_the_next_launch(monkeypatch):
    log = []

    def launch(name):
        log.append(("launch", name))
        return name

    def device(st):
        log.append(("device", st))

    def host(st):
        log.append(("host", st))
        return "metrics:" + st

    def stages_of(job):
        return (launch, device, host) if job.func is _staged else None

    monkeypatch.setattr(R, "_stages_of", stages_of)
    monkeypatch.setattr(R, "_table_fits_beside", lambda job: True)
    monkeypatch.setattr(R, "_launch_failed", lambda st: False)
    jobs = [functools.partial(_plain, log, "p0"), functools.partial(_staged, "a"),
            functools.partial(_staged, "b"), functools.partial(_staged, "c"),
            functools.partial(_plain, log, "p1"), functools.partial(_staged, "d")]
    out = R._run_jobs_pipelined(jobs)
    assert out == ["p0", "metrics:a", "metrics:b", "metrics:c", "p1", "metrics:d"]
    assert log == [("job", "p0"),
                   ("launch", "a"), ("device", "a"),
                   ("launch", "b"), ("host", "a"), ("device", "b"),
                   ("launch", "c"), ("host", "b"), ("device", "c"),
                   ("host", "c"), ("job", "p1"),
                   ("launch", "d"), ("device", "d"), ("host", "d")]


def test_staged_jobs_do_not_overlap_without_device_memory(monkeypatch):
    """overlapping holds two tables on the device.  A job whose table does not fit
    beside the held one runs after that job's host stage; a launch that fails beside it (out of
    memory) runs again once the held table's host stage is done."""
    log = []
    fails = {"c": 1}  # c's first launch fails

    def launch(name):
        log.append(("launch", name))
        if fails.get(name):
            fails[name] -= 1
            return "failed:" + name
        return name

    def device(st):
        log.append(("device", st))

    def host(st):
        log.append(("host", st))
        return "metrics:" + st

    monkeypatch.setattr(R, "_stages_of", lambda job: (launch, device, host)
                        if job.func is _staged else None)
    monkeypatch.setattr(R, "_table_fits_beside", lambda job: job.args[0] != "b")
    monkeypatch.setattr(R, "_launch_failed", lambda st: st.startswith("failed:"))
    jobs = [functools.partial(_staged, n) for n in "abcd"]
    out = R._run_jobs_pipelined(jobs)
    assert out == ["metrics:a", "metrics:b", "metrics:c", "metrics:d"]
    assert log == [("launch", "a"), ("device", "a"),
                   ("host", "a"), ("launch", "b"), ("device", "b"),       # b does not fit beside a
                   ("launch", "c"), ("host", "b"), ("launch", "c"),       # c failed beside b
                   ("device", "c"),
                   ("launch", "d"), ("host", "c"), ("device", "d"), ("host", "d")]


def test_launch_failed_reads_both_staged_job_kinds():
    assert R._launch_failed((None,) * 8)
    assert not R._launch_failed((None,) * 6 + (object(), None))
    assert R._launch_failed((object(), None, ValueError("x")))
    assert not R._launch_failed((object(), object(), None))


def test_histogram_scan_jobs_are_staged_only_without_state_io():
    from deequ_amd.analyzers import Histogram, Size
    plain = functools.partial(R._run_scanning_analyzers, None, [Histogram("x")], None, None)
    assert R._stages_of(plain) is not None
    for args in ([Histogram("x")], object(), None), ([Histogram("x")], None, object()), \
            ([Size()], None, None), ([Histogram("x"), Histogram("y")], None, None):
        job = functools.partial(R._run_scanning_analyzers, None, *args)
        assert R._stages_of(job) is None
