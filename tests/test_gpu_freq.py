"""GPU parity of the frequency path against the ORACLE (oracle/deequ_oracle.py `frequencies`,
restating GroupingAnalyzers.scala:53-80): the hash group-by, the shared aggregation over the table
(Uniqueness / Distinctness / UniqueValueRatio / CountDistinct / Entropy, AnalysisRunner.scala:
466-534), and the multi-GPU hash repartition -- P "ranks" are simulated in one
process on cuda:0: each shard's partial table is cut into P owner segments by the device kernels,
segment j of every source is handed to owner j exactly as the all-to-all would, and each owner
re-inserts what it received.  Bar: group counts bit-exact, every group on exactly one owner,
entropy within 1e-12 relative (north_star)."""
import math

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-12


def _table(n, seed, null_rate=0.05):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, max(1, n // 2), n)             # ~half the keys repeat
    ids[: min(3, n)] = np.iinfo(np.int64).min            # the exact-mode sentinel key
    words = np.array(["high", "low", "medium", "", "NullValue", "Thingy " + "q" * 30])
    s = words[rng.integers(0, len(words), n)]
    uniq = np.array([f"u{v}" for v in rng.integers(0, n, n)])
    def mask():
        return rng.random(n) < null_rate
    return pa.table({
        "id": pa.array(ids, mask=mask(), type=pa.int64()),
        "s": pa.array([None if m else v for v, m in zip(s, mask())], type=pa.string()),
        "u": pa.array([None if m else v for v, m in zip(uniq, mask())], type=pa.string()),
    })


def _otable(t):
    from oracle.deequ_oracle import OTable
    return OTable({k: t.column(k).to_pylist() for k in t.column_names},
                  {"id": "long", "s": "string", "u": "string"})


def _rel_close(a, b):
    return a == b or abs(a - b) <= REL * max(abs(a), abs(b))


@pytest.mark.parametrize("n,batch", [(1, None), (5000, None), (40_000, 8192)])
def test_frequency_family_matches_oracle(n, batch, gpu_device):
    from deequ_amd.analyzers import (CountDistinct, Distinctness, Entropy, UniqueValueRatio,
                                     Uniqueness)
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    t = _table(n, seed=n + 1)
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=batch)
    ot = _otable(t)
    # ("id", "s") mixes a fixed-width and a string key: AnalyzerTests.scala:87-94 pins
    # Uniqueness(Seq("unique", "nonUnique")) over such keys
    cases = [("id",), ("s",), ("u",), ("s", "u"), ("id", "s"), ("u", "id", "s")]
    analyzers = []
    for cols in cases:
        analyzers += [Uniqueness(cols), Distinctness(cols), UniqueValueRatio(cols),
                      CountDistinct(cols)]
    analyzers += [Entropy("id"), Entropy("s")]
    ctx = AnalysisRunner.do_analysis_run(df, analyzers)
    for cols in cases:
        freq = O.frequencies(ot, list(cols))
        exp = {Uniqueness(cols): O.uniqueness(freq, n), Distinctness(cols): O.distinctness(freq, n),
               UniqueValueRatio(cols): O.unique_value_ratio(freq),
               CountDistinct(cols): O.count_distinct(freq)}
        for a, v in exp.items():
            m = ctx.metric(a)
            if v is None:
                assert m.value.is_failure, str(a)
            else:
                assert m.value.get() == v, (str(a), m.value.get(), v)
    for col in ("id", "s"):
        v = O.entropy(O.frequencies(ot, [col]), n)
        got = ctx.metric(Entropy(col)).value.get()
        assert _rel_close(got, v), (col, got, v)


def _segments(rec, var, rc, vb):
    """Owner segment j of one source: (records bytes, var bytes)."""
    rb = 24
    r0 = np.concatenate([[0], np.cumsum(rc)]) * rb
    v0 = np.concatenate([[0], np.cumsum(vb)])
    return [(rec[int(r0[j]):int(r0[j + 1])], var[int(v0[j]):int(v0[j + 1])])
            for j in range(len(rc))]


def _repartition(t, cols, parts, device, null_as_group=False):
    """Simulated P-rank repartition on one device; returns the P owner tables."""
    import torch

    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.distributed import freq_add_records, freq_partition
    from deequ_amd.table import Table
    n = t.num_rows
    bounds = [n * r // parts for r in range(parts + 1)]
    sources, total_rows, special = [], 0, np.zeros(3, np.int64)
    types = None
    for r in range(parts):
        shard = Table.from_arrow(t.slice(bounds[r], bounds[r + 1] - bounds[r]), device=device)
        types = [shard.schema[c].dtype for c in cols]
        local = FrequencyTable(cols, types, 0)
        for b in shard.batches:
            local.add([b[c] for c in cols], null_as_group=null_as_group)
        total_rows += local.num_rows
        rec, var, rc, vb, sp = freq_partition(local, parts)
        special += sp
        sources.append((_segments(rec, var, rc, vb), rc, vb))
    owners = []
    for o in range(parts):
        recs = torch.cat([s[0][o][0] for s in sources])
        vars_ = torch.cat([s[0][o][1] for s in sources])
        src_rc = np.array([s[1][o] for s in sources], np.int64)
        src_vb = np.array([s[2][o] for s in sources], np.int64)
        owned = FrequencyTable(cols, types, 0)
        freq_add_records(owned, recs, vars_, src_rc, src_vb, total_rows,
                         special if o == 0 else np.zeros(3, np.int64), null_as_group)
        owners.append(owned)
    return owners


@pytest.mark.parametrize("parts", [1, 2, 3, 8])
@pytest.mark.parametrize("cols", [("id",), ("s",), ("u",), ("s", "u"), ("id", "s")])
def test_repartition_matches_single_table(parts, cols, gpu_device):
    from oracle import deequ_oracle as O
    n = 30_000
    t = _table(n, seed=7 * parts + len(cols))
    freq = O.frequencies(_otable(t), list(cols))
    owners = _repartition(t, list(cols), parts, gpu_device)
    seen = {}
    for owned in owners:
        assert owned.num_rows == n
        for key, cnt in owned.export():
            assert key not in seen, f"group {key} on two owners"
            seen[key] = cnt
    assert seen == freq
    g = u = 0
    e = 0.0
    for owned in owners:
        s = owned.summarize()
        g += s.n_groups
        u += s.n_unique
        e += s.entropy
    assert g == len(freq) and u == sum(1 for c in freq.values() if c == 1)
    assert _rel_close(e, O.entropy(freq, n))


@pytest.mark.parametrize("col", ["id", "s"])
def test_repartition_histogram_null_group(col, gpu_device):
    """Histogram mode (NULL is its own group, Histogram.scala:59-66) through the repartition: the
    NULL group stays apart from a real "NullValue" string (folded only when Histogram reads it)."""
    t = _table(20_000, seed=3, null_rate=0.1)
    vals = t.column(col).to_pylist()
    exp = {}
    for v in vals:
        exp[(v,)] = exp.get((v,), 0) + 1
    owners = _repartition(t, [col], 4, gpu_device, null_as_group=True)
    got = {}
    nullg = lit = 0
    for owned in owners:
        for key, cnt in owned.export():
            assert key not in got
            got[key] = cnt
        a, b = owned.null_literal()
        nullg, lit = nullg + a, lit + b
    assert got == exp
    assert nullg == exp[(None,)]
    assert lit == (exp.get(("NullValue",), 0) if col == "s" else 0)


@pytest.mark.parametrize("cols", [("id",), ("s",)])
def test_reset_table_equals_fresh_table(cols, gpu_device):
    """dq_freq_reset keeps capacity but no groups, counters or numRows."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    t1, t2 = _table(20_000, seed=91), _table(7_000, seed=92)
    d1, d2 = Table.from_arrow(t1, device=gpu_device), Table.from_arrow(t2, device=gpu_device)
    types = [d1.schema[c].dtype for c in cols]
    ft = FrequencyTable(list(cols), types, 0, capacity_hint=20_000)
    for b in d1.batches:
        ft.add([b[c] for c in cols])
    ft.reset()
    for b in d2.batches:
        ft.add([b[c] for c in cols])
    assert ft.num_rows == 7_000
    assert dict(ft.export()) == O.frequencies(_otable(t2), list(cols))


def _freq_table(t, cols, device, null_as_group=False):
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    df = Table.from_arrow(t, device=device, max_batch_rows=7_000)
    ft = FrequencyTable(list(cols), [df.schema[c].dtype for c in cols], 0)
    for b in df.batches:
        ft.add([b[c] for c in cols], null_as_group=null_as_group)
    return ft


@pytest.mark.parametrize("cols", [("id",), ("s",), ("u",), ("s", "u"), ("id", "s")])
def test_merged_tables_equal_whole_table(cols, gpu_device):
    """FrequenciesAndNumRows.sum (GroupingAnalyzers.scala:128-148) on the device: random row
    splits, one table per part, merged with dq_freq_merge == the whole table (counts, numRows)."""
    from oracle import deequ_oracle as O
    n = 25_000
    t = _table(n, seed=41 + len(cols))
    rng = np.random.default_rng(len(cols))
    cuts = sorted(rng.choice(np.arange(1, n), 3, replace=False).tolist())
    bounds = [0] + cuts + [n]
    parts = [_freq_table(t.slice(bounds[i], bounds[i + 1] - bounds[i]), cols, gpu_device)
             for i in range(len(bounds) - 1)]
    merged = parts[0]
    for p in parts[1:]:
        merged = merged.merged(p)
    assert merged.num_rows == n
    freq = O.frequencies(_otable(t), list(cols))
    assert dict(merged.export()) == freq
    s = merged.summarize()
    assert s.n_groups == len(freq) and s.n_unique == sum(1 for c in freq.values() if c == 1)
    assert _rel_close(s.entropy, O.entropy(freq, n))


def test_merge_keeps_hash_collisions_apart_and_handles_histogram_nulls(gpu_device):
    """Histogram tables (NULL group) merge; a string table merged with itself doubles counts."""
    t = _table(12_000, seed=5, null_rate=0.2)
    for col in ("id", "s"):
        a = _freq_table(t, [col], gpu_device, null_as_group=True)
        b = _freq_table(t, [col], gpu_device, null_as_group=True)
        m = a.merged(b)
        got = dict(m.export())
        exp = {}
        for v in t.column(col).to_pylist():
            exp[(v,)] = exp.get((v,), 0) + 2
        assert got == exp, col
        assert m.null_literal() == (exp[(None,)], exp.get(("NullValue",), 0) if col == "s" else 0)


@pytest.mark.parametrize("n,k", [(1, 10), (5000, 3), (3000, 2000), (40_000, 1000), (200_000, 1000)])
@pytest.mark.parametrize("col", ["id", "s", "u"])
def test_topk_matches_oracle_order(n, k, col, gpu_device):
    """dq_freq_topk == rdd.top(k)(OrderByAbsoluteCount) up to ties: the multiset of returned counts
    is the oracle's k largest, and every returned key carries its exact count.  Raw table: the
    NULL group apart; Histogram's view (_fold_null_group): NULL folded into "NullValue"."""
    from deequ_amd import _native as N
    from deequ_amd.analyzers.grouping import _fold_null_group, cast_to_string
    t = _table(n, seed=n + 3)
    ft = _freq_table(t, [col], gpu_device, null_as_group=True)
    got = ft.topk(k)
    vals = t.column(col).to_pylist()
    raw, exp = {}, {}
    for v in vals:
        raw[v] = raw.get(v, 0) + 1
        f = "NullValue" if v is None and col != "id" else v
        exp[f] = exp.get(f, 0) + 1
    assert [c for _, c in got] == sorted(raw.values(), reverse=True)[:k]
    for (key,), c in got:
        assert raw[key] == c
    assert ft.count() == len(raw)
    dtype = N.INT64 if col == "id" else N.UTF8
    top, bins = _fold_null_group(ft, dtype, k)
    assert bins == len(exp)
    assert [c for _, c in top] == sorted(exp.values(), reverse=True)[:k]
    str_exp = {cast_to_string(key, dtype): c for key, c in exp.items()}
    for key, c in top:
        assert str_exp[key] == c


@pytest.mark.parametrize("target", ["1", "7", "1000000000"])
def test_partition_depths_and_recount(target, gpu_device, monkeypatch):
    """The partition sizing at both extremes: target 1 drives s to its maximum (10 sub-bucket
    bits) on a small table, and a huge target keeps s = 0 so that 600K distinct keys overflow the
    512 partitions' LDS tables and take the recount path.  Results must not change."""
    from oracle import deequ_oracle as O
    monkeypatch.setenv("DQ_FREQ_PARTITION_TARGET", target)
    n = 600_000 if target == "1000000000" else 60_000
    rng = np.random.default_rng(int(target) % 97)
    ids = rng.permutation(n).astype(np.int64)
    ids[: n // 10] = ids[n // 10: n // 5]          # some repeats
    words = np.array([f"w{v}" for v in ids])
    t = pa.table({"id": pa.array(ids), "s": pa.array(words)})
    for cols in (("id",), ("s",)):
        ft = _freq_table(t, list(cols), gpu_device)
        s = ft.summarize()
        exp = {}
        for v in t.column(cols[0]).to_pylist():
            exp[v] = exp.get(v, 0) + 1
        assert s.n_groups == len(exp)
        assert s.n_unique == sum(1 for c in exp.values() if c == 1)
        got = {k[0]: c for k, c in ft.export()}
        assert got == exp
        top = ft.topk(5)
        assert [c for _, c in top] == sorted(exp.values(), reverse=True)[:5]


@pytest.mark.parametrize("heavy", [0.02, 0.3])
def test_packed_phase_c_hands_on_heavy_partitions(heavy, gpu_device, monkeypatch):
    """Exact mode partitioned to the full depth (s = 10) counts in packed slots (count << 45 |
    key); a partition holding a record whose count is >= 128 (a heavy key collapsed in phase A)
    or more than 4096 records is handed on whole to the two-word kernel.  Mixed heavy keys and
    unique keys must give the oracle's groups, statistics and top-k either way."""
    monkeypatch.setenv("DQ_FREQ_PARTITION_TARGET", "1")
    n = 200_000
    rng = np.random.default_rng(5)
    ids = rng.permutation(n).astype(np.int64) * 3
    hv = rng.random(n) < heavy
    ids[hv] = rng.choice(np.array([7, 11, 13], dtype=np.int64), size=int(hv.sum()))
    t = pa.table({"id": pa.array(ids)})
    ft = _freq_table(t, ["id"], gpu_device)
    exp = {}
    for v in ids.tolist():
        exp[v] = exp.get(v, 0) + 1
    s = ft.summarize()
    assert s.n_groups == len(exp)
    assert s.n_unique == sum(1 for c in exp.values() if c == 1)
    ent = -math.fsum((c / n) * math.log(c / n) for c in exp.values())
    assert abs(s.entropy - ent) <= 1e-12 * abs(ent)
    top = ft.topk(6)
    assert [c for _, c in top] == sorted(exp.values(), reverse=True)[:6]
    for (key,), c in top:
        assert exp[key] == c
    assert {k[0]: c for k, c in ft.export()} == exp


@pytest.mark.parametrize("kind,target", [("long", None), ("long", "50"), ("string", None),
                                         ("string", "50")])
def test_topk_recounts_only_partitions_that_may_hold_outranking_groups(kind, target, gpu_device,
                                                                        monkeypatch):
    """dq_freq_topk with a flat count distribution (many groups of similar counts, so partitions
    hold more groups than their listed candidates): the partitions whose unlisted groups could
    outrank the selection are counted again with their groups, and the top k come from the
    other partitions' candidates plus those groups.  Bar: the oracle's top-k counts and each
    returned key's count, the same as the exact path (DQ_FREQ_TOPK_EXACT=1)."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    if target:
        monkeypatch.setenv("DQ_FREQ_PARTITION_TARGET", target)
    rng = np.random.default_rng(3 if kind == "long" else 4)
    g = 60_000
    cnt = rng.integers(1, 41, g)
    keys = rng.permutation(g).astype(np.int64) * 13 + 5
    ids = rng.permutation(np.repeat(keys, cnt))
    col = pa.array(ids) if kind == "long" else pa.array([f"k{v}" for v in ids.tolist()])
    df = Table.from_arrow(pa.table({"c": col}), device=gpu_device, max_batch_rows=1 << 20)

    def top(k):
        ft = FrequencyTable(["c"], [df.schema["c"].dtype], 0)
        for b in df.batches:
            ft.add([b["c"]])
        return ft.topk(k)
    exp = dict(zip(keys.tolist(), cnt.tolist()))
    if kind == "string":
        exp = {f"k{v}": c for v, c in exp.items()}
    for k in (1000, 10):
        got = top(k)
        assert [c for _, c in got] == sorted(exp.values(), reverse=True)[:k]
        for (key,), c in got:
            assert exp[key] == c
    monkeypatch.setenv("DQ_FREQ_TOPK_EXACT", "1")
    assert [c for _, c in top(1000)] == sorted(exp.values(), reverse=True)[:1000]


@pytest.mark.parametrize("target", ["100", "45", "20", "4"])  # s = 7, 8, 9, 10 sub-bits
def test_packed_slots_mixed_counts_of_one_key(target, gpu_device, monkeypatch):
    """Packed phase-C slots (s = 7..10 sub-bits) with one key arriving as records of different
    counts in one partition (a run of the key collapsed in phase A's LDS table, plus a single
    copy elsewhere): every record of a key must probe the same slot sequence (the double-hashing
    step comes from key bits, never from the count field), or a key splits into two groups.
    Bar: the oracle's group count, unique count, entropy and top counts."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    monkeypatch.setenv("DQ_FREQ_PARTITION_TARGET", target)
    rng = np.random.default_rng(int(target))
    keys = rng.permutation(3_000_000).astype(np.int64) * 7 + 1
    runs = rng.integers(1, 4, len(keys))
    ids = np.repeat(keys, runs)
    extra = rng.choice(keys, 1_000_000, replace=False)
    ids = np.concatenate([ids, extra])
    df = Table.from_arrow(pa.table({"id": pa.array(ids)}), device=gpu_device, max_batch_rows=1 << 21)
    ft = FrequencyTable(["id"], [df.schema["id"].dtype], 0)
    for b in df.batches:
        ft.add([b["id"]])
    _, cnt = np.unique(ids, return_counts=True)
    s = ft.summarize()
    assert s.n_groups == len(cnt)
    assert s.n_unique == int((cnt == 1).sum())
    n = len(ids)
    ent = -math.fsum(((cnt / n) * np.log(cnt / n)).tolist())
    assert abs(s.entropy - ent) <= 1e-12 * abs(ent)
    top = ft.topk(8)
    assert [c for _, c in top] == sorted(cnt.tolist(), reverse=True)[:8]


@pytest.mark.parametrize("col,nulls", [("id", 0.05), ("id", 0.0), ("s", 0.0)])
def test_histogram_table_serves_grouping(col, nulls, gpu_device):
    """The runner groups a column once for Histogram(col) and its grouping analyzers when
    Histogram.table_serves_grouping holds: the keyed view of the Histogram-mode table
    (dq_freq_summarize_keys) must equal the grouping table bit for bit, and the metrics of the
    shared run must equal the oracle's."""
    from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
    from deequ_amd.analyzers.grouping import KeyedFrequencies
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    n = 30_000
    t = _table(n, seed=77, null_rate=nulls)
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=7_000)
    assert Histogram.table_serves_grouping(df, col)
    grouping = _freq_table(t, [col], gpu_device)
    keyed = KeyedFrequencies(_freq_table(t, [col], gpu_device, null_as_group=True))
    a, b = grouping.summarize(), keyed.summarize()
    for f in ("num_rows", "n_groups", "n_unique", "n_null_key_rows"):
        assert getattr(a, f) == getattr(b, f), f
    assert a.entropy == b.entropy
    assert dict(keyed.export()) == dict(grouping.export())
    assert keyed.count() == grouping.count()
    suite = [Uniqueness([col]), Distinctness([col]), Entropy(col), Histogram(col)]
    ctx = AnalysisRunner.do_analysis_run(df, suite)
    freq = O.frequencies(_otable(t), [col])
    assert ctx.metric(Uniqueness([col])).value.get() == O.uniqueness(freq, n)
    assert ctx.metric(Distinctness([col])).value.get() == O.distinctness(freq, n)
    assert _rel_close(ctx.metric(Entropy(col)).value.get(), O.entropy(freq, n))
    hist = ctx.metric(Histogram(col)).value.get()
    exp_bins = len(freq) + (1 if nulls and col == "id" else 0)
    assert hist.number_of_bins == exp_bins


@pytest.mark.parametrize("k", [1, 2, 1000])
def test_histogram_shares_string_table_with_grouping(k, gpu_device):
    """Histogram("s") and the grouping of ["s"] read ONE group-by of a string column with NULLs
    and real "NullValue" strings (runners._histogram_columns_for_groupings): the grouping drops the
    NULL rows (GroupingAnalyzers.scala:62-65), Histogram folds them into "NullValue"
    (Histogram.scala:59-66) -- both equal to the oracle's."""
    from deequ_amd.analyzers import CountDistinct, Entropy, Histogram, Uniqueness
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    n = 30_000
    t = _table(n, seed=77, null_rate=0.3)   # NULL rows outnumber every string: the fold ranks first
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=8192)
    ot = _otable(t)
    h = Histogram("s", max_detail_bins=k)
    ctx = AnalysisRunner.do_analysis_run(df, [h, Uniqueness(["s"]), Entropy("s"), CountDistinct(["s"])])
    freq = O.frequencies(ot, ["s"])
    assert ctx.metric(Uniqueness(["s"])).value.get() == O.uniqueness(freq, n)
    assert ctx.metric(CountDistinct(["s"])).value.get() == O.count_distinct(freq)
    assert _rel_close(ctx.metric(Entropy("s")).value.get(), O.entropy(freq, n))
    hist, _ = O.histogram(ot, "s")
    dist = ctx.metric(h).value.get()
    assert dist.number_of_bins == len(hist)
    want = sorted(hist.values(), reverse=True)[:k]
    got = sorted((v.absolute for v in dist.values.values()), reverse=True)
    assert got == want
    for key, v in dist.values.items():
        assert hist[key] == v.absolute and v.ratio == v.absolute / n


@pytest.mark.parametrize("distinct", [40, 5000])
def test_short_string_keys_of_every_length(distinct, gpu_device):
    """One utf8 key column whose values have every length 0..24, embedded NUL bytes and shared
    prefixes ("a", "a\\0", "a\\0\\0", ...): the branch-free hash of strings <= 16 bytes, the
    short-key LDS comparisons and the batched first probe of the one-string phase A must keep
    every distinct string its own group.  60k rows span many phase-A tiles per workgroup, so the
    low-cardinality case runs the non-probing tiles' fast path.  Bar: exported frequencies equal
    the oracle's exactly."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(distinct)
    base = ["", "a", "a\x00", "a\x00\x00", "\x00", "\x00a", "ab" * 4, "ab" * 4 + "\x00",
            "x" * 15, "x" * 16, "x" * 17, "y" * 24, "NullValue"]
    vocab = list(base)
    while len(vocab) < distinct:
        k = int(rng.integers(0, 25))
        vocab.append("".join(chr(int(c)) for c in rng.integers(0, 3, k)))  # bytes 0..2
    vocab = sorted(set(vocab))
    n = 60_000
    vals = [vocab[i] for i in rng.integers(0, len(vocab), n)]
    mask = rng.random(n) < 0.03
    t = pa.table({"s": pa.array([None if m else v for v, m in zip(vals, mask)],
                                type=pa.string())})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=1 << 14)
    ft = FrequencyTable(["s"], [df.schema["s"].dtype], 0, capacity_hint=n)
    for b in df.batches:
        ft.add([b["s"]])
    ot = O.OTable({"s": t.column("s").to_pylist()}, {"s": "string"})
    assert dict(ft.export()) == O.frequencies(ot, ["s"])
    assert ft.num_rows == n


@pytest.mark.parametrize("distinct,poison", [(1, None), (3, None), (8, None), (3, "long"),
                                             (12, None), (3, "late_long")])
@pytest.mark.parametrize("nulls", [0.0, 0.1])
def test_small_key_phase_a_matches_oracle(distinct, poison, nulls, gpu_device):
    """One utf8 key of strings <= 7 bytes with few values (freq_phaseA_small: exact packed keys,
    per-lane counters).  8 values fit a wave's candidates; 12 do not, and a string longer than 7
    bytes anywhere in a batch ("long": mid-table, "late_long": the last rows of the last batch)
    makes the kernel give that batch up to the general phase A -- batches before it keep the small
    kernel's output.  Empty strings, embedded NULs and a ragged last batch included.  Bar: the
    grouping's frequencies and the Histogram / grouping metrics of a shared run equal the
    oracle's."""
    from deequ_amd.analyzers import CountDistinct, Entropy, Histogram, Uniqueness
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(distinct * 7 + (poison is not None))
    vocab = ["", "a", "a\x00", "\x00", "high", "low", "medium", "zzzzzzz", "b\x00\x00c",
             "q1", "q2", "q3"][:distinct]
    n = 200_003
    vals = [vocab[i] for i in rng.integers(0, len(vocab), n)]
    if poison == "long":
        vals[100_000] = "eight+1ch"
    elif poison == "late_long":
        vals[n - 3] = "a much longer string"
    mask = rng.random(n) < nulls
    t = pa.table({"s": pa.array([None if m else v for v, m in zip(vals, mask)], pa.string())})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=1 << 16)
    assert len(df.batches) == 4
    ot = O.OTable({"s": t.column("s").to_pylist()}, {"s": "string"})
    freq = O.frequencies(ot, ["s"])
    ft = FrequencyTable(["s"], [df.schema["s"].dtype], 0, capacity_hint=n)
    for b in df.batches:
        ft.add([b["s"]])
    assert dict(ft.export()) == freq
    assert ft.num_rows == n
    h = Histogram("s")
    ctx = AnalysisRunner.do_analysis_run(df, [h, Uniqueness(["s"]), Entropy("s"),
                                              CountDistinct(["s"])])
    assert ctx.metric(Uniqueness(["s"])).value.get() == O.uniqueness(freq, n)
    assert ctx.metric(CountDistinct(["s"])).value.get() == O.count_distinct(freq)
    assert _rel_close(ctx.metric(Entropy("s")).value.get(), O.entropy(freq, n))
    hist, _ = O.histogram(ot, "s")
    dist = ctx.metric(h).value.get()
    assert dist.number_of_bins == len(hist)
    assert {k: v.absolute for k, v in dist.values.items()} == hist


def test_small_key_phase_a_on_unaligned_and_sliced_batches(gpu_device):
    """The small-key kernel's bounds-checked path: a batch whose validity bitmap is not dword
    aligned (a row slice of a device table, 8 rows in) and whose length is not a multiple of the
    1024-row step."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(5)
    vocab = ["x", "yy", "", "zzz"]
    n = 70_001
    vals = [None if rng.random() < 0.05 else vocab[i] for i in rng.integers(0, 4, n)]
    t = pa.table({"s": pa.array(vals, pa.string())})
    df = Table.from_arrow(t, device=gpu_device).select_rows(8, n - 5)
    ft = FrequencyTable(["s"], [df.schema["s"].dtype], 0)
    for b in df.batches:
        ft.add([b["s"]])
    ot = O.OTable({"s": vals[8:n - 5]}, {"s": "string"})
    assert dict(ft.export()) == O.frequencies(ot, ["s"])


def test_small_key_batch_table_overflow(gpu_device):
    """freq_phaseA_small merges the workgroups' groups in a 64-slot device table per batch; keys
    beyond its capacity stay in the workgroups' own records (and the last workgroup to arrive writes
    the table's).  Rows draw from 5 keys of a window that moves every 30720 rows (one workgroup's
    range), so every wave stays within its 8 candidates while the batch holds ~170 distinct keys.
    Bar: frequencies and Histogram equal the oracle's."""
    from deequ_amd.analyzers import Histogram
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(17)
    n = 1 << 20
    region = np.arange(n) // 30720
    pick = region * 5 + rng.integers(0, 5, n)
    vals = [None if rng.random() < 0.02 else f"k{p:03d}" for p in pick.tolist()]
    t = pa.table({"s": pa.array(vals, pa.string())})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=1 << 19)
    ft = FrequencyTable(["s"], [df.schema["s"].dtype], 0, capacity_hint=n)
    for b in df.batches:
        ft.add([b["s"]])
    ot = O.OTable({"s": vals}, {"s": "string"})
    freq = O.frequencies(ot, ["s"])
    assert len(freq) > 64
    assert dict(ft.export()) == freq
    ctx = AnalysisRunner.do_analysis_run(df, [Histogram("s")])
    hist, _ = O.histogram(ot, "s")
    dist = ctx.metric(Histogram("s")).value.get()
    assert dist.number_of_bins == len(hist)
    assert {k: v.absolute for k, v in dist.values.items()} == hist


@pytest.mark.parametrize("nulls", [0.0, 0.05])
def test_exact_bucket_pieces_at_scale(nulls, gpu_device):
    """12M int64 rows in 4M-row batches: bucket pieces from several batches and workgroups
    (freq_prepass_x + freq_phaseA_xp), several phase-B units per bucket and per persistent B3
    workgroup, full-depth partitions (s = 10) in packed phase C -- against numpy's exact counts
    and the C restatement's entropy."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    n = 12_000_000
    rng = np.random.default_rng(11)
    ids = rng.integers(0, 9_000_000, n, dtype=np.int64)      # ~26 % of keys repeated
    ids[:2000] = 42                                           # one heavy key (collapses in A)
    mask = rng.random(n) < nulls
    t = pa.table({"id": pa.array(ids, mask=mask)})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=4_000_000)
    ft = FrequencyTable(["id"], [df.schema["id"].dtype], 0)
    for b in df.batches:
        ft.add([b["id"]])
    s = ft.summarize()
    vals, counts = np.unique(ids[~mask], return_counts=True)
    assert s.num_rows == n
    assert s.n_groups == len(vals)
    assert s.n_unique == int((counts == 1).sum())
    p = counts / n
    ent = -math.fsum((p * np.log(p)).tolist())
    assert abs(s.entropy - ent) <= 1e-12 * abs(ent)
    top = ft.topk(3)
    order = np.argsort(-counts, kind="stable")[:3]
    assert [c for _, c in top] == counts[order].tolist()
    assert top[0][0][0] == 42


@pytest.mark.parametrize("scale,heavy", [("1", 0), ("1", 400), ("0.5", 0), ("0.97", 0)])
def test_capacity_layout_and_its_counted_fallback(scale, heavy, gpu_device, monkeypatch):
    """Exact phase B without the count pass (finalize_b's capacity layout): partitions of fixed
    room filled through cursor adds.  DQ_FREQ_CAP_SCALE shrinks the room so runs overflow and the
    table is scattered again by the counted path (0.5: every partition; 0.97: a few); `heavy`
    keys repeated once per 8192-row tile bypass phase A's dedupe and crowd one partition.  Every
    case against numpy's exact counts, the entropy within 1e-12, and the top 3."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    monkeypatch.setenv("DQ_FREQ_CAP_SCALE", scale)
    n = 6_000_000
    rng = np.random.default_rng(5)
    ids = rng.integers(-2**62, 2**62, n, dtype=np.int64)     # distinct: the dedupe bypasses
    if heavy:
        ids[::8192][:heavy] = 7                                  # one key in every tile
    t = pa.table({"id": pa.array(ids)})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=2_000_000)
    ft = FrequencyTable(["id"], [df.schema["id"].dtype], 0)
    for b in df.batches:
        ft.add([b["id"]])
    s = ft.summarize()
    vals, counts = np.unique(ids, return_counts=True)
    assert s.num_rows == n
    assert s.n_groups == len(vals)
    assert s.n_unique == int((counts == 1).sum())
    p = counts / n
    ent = -math.fsum((p * np.log(p)).tolist())
    assert abs(s.entropy - ent) <= 1e-12 * abs(ent)
    top = ft.topk(3)
    assert [c for _, c in top][:1] == [int(counts.max())]
    if heavy:
        assert top[0][0][0] == 7


@pytest.mark.parametrize("batch", [None, 9_000])
def test_long_string_keys_match_oracle(batch, gpu_device):
    """One-column and two-column keys over strings of 17..80 bytes (the chunked long-string hash:
    the device's register path up to 48 bytes, 16 bytes per round beyond), with duplicates within
    and across batches, and a merge of two tables: groups, Σ[c==1] and entropy vs the oracle."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(21)
    n = 30_000
    base = [("https://example.org/" * 4)[: rng.integers(17, 81)] for _ in range(40)]
    keys = [base[i % 40][:-3] + f"{rng.integers(0, 300):03d}" for i in range(n)]
    mask = rng.random(n) < 0.04
    t = pa.table({"l": pa.array([None if m else k for k, m in zip(keys, mask)], pa.string()),
                  "p": pa.array([["a", "bb", None][i % 3] for i in range(n)], pa.string())})
    ot = O.OTable({"l": t.column("l").to_pylist(), "p": t.column("p").to_pylist()},
                  {"l": "string", "p": "string"})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=batch)
    for cols in (["l"], ["l", "p"]):
        exp = O.frequencies(ot, cols)
        nb = len(df.batches)
        cuts = ((0, nb // 2), (nb // 2, nb)) if nb > 1 else ((0, nb),)
        halves = []
        for lo, hi in cuts:
            ft = FrequencyTable(cols, [df.schema[c].dtype for c in cols], 0)
            for b in df.batches[lo:hi]:
                ft.add([b[c] for c in cols])
            halves.append(ft)
        ft = halves[0].merged(halves[1]) if len(halves) > 1 else halves[0]
        s = ft.summarize()
        assert s.n_groups == len(exp)
        assert s.n_unique == sum(1 for c in exp.values() if c == 1)
        assert dict(ft.export()) == exp
        ent = O.entropy(exp, n)
        assert _rel_close(s.entropy, ent)


@pytest.mark.parametrize("long_frac", [0.0, 0.01])
def test_two_small_string_columns_dedupe_on_short_forms(long_frac, gpu_device):
    """A two-column utf8 key whose values are at most 7 bytes (a MutualInformation joint of two
    low-cardinality columns) dedupes in phase A on its LDS short form; a few longer values take
    the row compare.  Groups, Σ[c==1] and entropy vs the oracle."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(5)
    n = 200_000
    pa_vals = np.array(["high", "low", "medium", "", "x"], dtype=object)
    pb_vals = np.array(["a", "bb", "ccc", "dddd", "eeeeeee"], dtype=object)
    a_ = pa_vals[rng.integers(0, 5, n)]
    b_ = pb_vals[rng.integers(0, 5, n)]
    longs = rng.random(n) < long_frac
    b_ = np.where(longs, "a much longer value", b_)
    ma, mb = rng.random(n) < 0.05, rng.random(n) < 0.05
    t = pa.table({"a": pa.array([None if m else v for v, m in zip(a_, ma)], pa.string()),
                  "b": pa.array([None if m else v for v, m in zip(b_, mb)], pa.string())})
    ot = O.OTable({"a": t.column("a").to_pylist(), "b": t.column("b").to_pylist()},
                  {"a": "string", "b": "string"})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=50_000)
    ft = FrequencyTable(["a", "b"], [df.schema["a"].dtype, df.schema["b"].dtype], 0)
    for b in df.batches:
        ft.add([b["a"], b["b"]])
    exp = O.frequencies(ot, ["a", "b"])
    s = ft.summarize()
    assert s.n_groups == len(exp)
    assert s.n_unique == sum(1 for c in exp.values() if c == 1)
    assert dict(ft.export()) == exp
    assert _rel_close(s.entropy, O.entropy(exp, n))


def test_large_export_reads_back_past_the_pinned_staging(gpu_device):
    """An export of 3.2M groups (77 MB of records) takes d2h's plain-copy path (blocks over 64 MB
    are not staged through pinned memory); every group and count must come back."""
    rng = np.random.default_rng(77)
    n = 3_400_000
    ids = rng.permutation(np.arange(n, dtype=np.int64) * 7919)[: 3_200_000]
    ids = np.concatenate([ids, ids[:200_000]])  # 200k keys twice
    t = pa.table({"id": pa.array(ids, type=pa.int64())})
    ft = _freq_table(t, ["id"], gpu_device)
    got = dict(ft.export())
    keys, counts = np.unique(ids, return_counts=True)
    assert len(got) == len(keys)
    assert sum(got.values()) == len(ids)
    exp = dict(zip(keys.tolist(), counts.tolist()))
    assert got == {(k,): c for k, c in exp.items()}


def test_many_small_key_tables_reuse_pinned_words(gpu_device):
    """More tables than one pinned block holds (512 small-key flag words), each created,
    filled through the small-key path and destroyed: every one counts its groups right."""
    from deequ_amd.analyzers.grouping import _fold_null_group
    from deequ_amd import _native as N
    rng = np.random.default_rng(5)
    n = 5000
    words = np.array(["a", "bb", "ccc", "dd"])
    for i in range(600):
        v = words[rng.integers(0, len(words) - (i % 2), n)]
        mask = rng.random(n) < 0.1
        t = pa.table({"s": pa.array([None if m else x for x, m in zip(v, mask)], pa.string())})
        ft = _freq_table(t, ["s"], gpu_device, null_as_group=True)
        top, bins = _fold_null_group(ft, N.UTF8, 10)
        exp = {}
        for x, m in zip(v, mask):
            k = "NullValue" if m else x
            exp[k] = exp.get(k, 0) + 1
        assert dict(top) == exp and bins == len(exp), i
        del ft


@pytest.mark.gpu
@pytest.mark.parametrize("offset", [0, 3])
def test_two_string_columns_all_length_classes(offset, gpu_device):
    """Two utf8 key columns (MutualInformation joints of string columns) take phase A's
    two-column path: both values' offsets and <= 16 bytes loaded as aligned dwords for two rounds
    at once, the row hash and encoding from registers.  Values of every length class (empty,
    <= 7 bytes: short keys, 8..16, > 16: the long hash and byte encoding), NULLs in either column,
    high cardinality (most rows go to the arena raw) and sliced batches: the groups, Σ[c==1] and
    the entropy vs the oracle."""
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    rng = np.random.default_rng(41 + offset)
    n = 150_000 + offset
    stems = ["", "q", "abcdefg", "abcdefgh", "0123456789abcdef", "a value over sixteen bytes",
             "x" * 40]

    def col(card):
        v = rng.integers(0, card, n)
        s = rng.integers(0, len(stems), n)
        m = rng.random(n) < 0.05
        return pa.array([None if mm else (stems[ss] + (str(vv) if ss else ""))[: 60]
                         for vv, ss, mm in zip(v, s, m)], pa.string())
    a, b = col(40_000), col(30)
    t = pa.table({"a": a, "b": b}).slice(offset)
    ot = O.OTable({"a": t.column("a").to_pylist(), "b": t.column("b").to_pylist()},
                  {"a": "string", "b": "string"})
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=37_000)
    ft = FrequencyTable(["a", "b"], [df.schema["a"].dtype, df.schema["b"].dtype], 0)
    for bt in df.batches:
        ft.add([bt["a"], bt["b"]])
    exp = O.frequencies(ot, ["a", "b"])
    s = ft.summarize()
    assert s.n_groups == len(exp)
    assert s.n_unique == sum(1 for c in exp.values() if c == 1)
    assert dict(ft.export()) == exp
    # (~1e5 groups: the oracle's running sum drifts by ~1e-12; the terms summed exactly instead)
    m = t.num_rows
    assert _rel_close(s.entropy, math.fsum(-(c / m) * math.log(c / m) for c in exp.values()))
