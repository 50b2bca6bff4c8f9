"""Generates tests/golden/vectors.json: golden input/output vectors for the hot path (SURVEY.md
§8(c) items ii-v), computed by the CPU restatement in oracle/deequ_oracle.py.

    python tests/golden/make_golden.py

The reference (Scala on Spark 2.2) cannot run in this image (no JVM), so the
vectors come from the oracle, which is itself pinned by the reference's known answers
(reference_known_answers.json) and by the independent `xxhash` package for XXH64.  Inputs are
not stored: tests/golden_inputs.py regenerates them bit-identically from (n, seed, null_rate)
with numpy's PCG64.  Floats are stored as JSON numbers (repr round-trips exactly); NaN as NaN.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.dirname(HERE)]

from golden_inputs import (CASES, FREQ_COLS, SCAN_AGGS, TYPES, XXH_INPUTS,  # noqa: E402
                           golden_table)


def oracle_table(t):
    from oracle.deequ_oracle import OTable
    return OTable({k: t.column(k).to_pylist() for k in t.column_names}, TYPES)


def scan_expected(ot, kind, arg, where):
    from oracle import deequ_oracle as O
    if kind == "count":
        return O.agg_count_all(ot) if where is None else O.agg_conditional_count(ot, where)
    if kind == "notnull":
        return O.agg_sum_notnull(ot, arg, where)
    if kind == "compliance":
        return O.agg_compliance(ot, arg, where)
    if kind == "sum":
        return O.agg_sum(ot, arg, where)
    if kind == "min":
        return O.agg_min(ot, arg, where)
    if kind == "max":
        return O.agg_max(ot, arg, where)
    if kind == "stddev":
        return list(O.agg_stddev(ot, arg, where))
    if kind == "corr":
        return list(O.agg_corr(ot, arg[0], arg[1], where))
    if kind == "hll":
        words = O.agg_hll(ot, arg, where)
        est, corrected = O.hll_count(words)
        return {"words": [int(w) for w in words], "estimate": est, "bias_corrected": corrected}
    raise ValueError(kind)


def freq_expected(ot, cols):
    from oracle import deequ_oracle as O
    f = O.frequencies(ot, cols)
    n = ot.n
    counts = sorted(f.values())
    return {
        "num_rows": n,
        "groups": len(f),
        "count_sum": sum(counts),
        "singletons": sum(1 for c in counts if c == 1),
        "max_count": counts[-1] if counts else 0,
        "uniqueness": O.uniqueness(f, n),
        "distinctness": O.distinctness(f, n),
        "unique_value_ratio": O.unique_value_ratio(f),
        "count_distinct": O.count_distinct(f),
        "entropy": O.entropy(f, n),
    }


def histogram_expected(ot, col):
    from oracle import deequ_oracle as O
    h, n = O.histogram(ot, col)
    return {"num_rows": n, "bins": len(h), "counts": {k: v for k, v in sorted(h.items())}}


# int64 values whose XXH64 (seed 42) has HLL++ rank 31..39 (found by
# tools/find_high_rank_longs.c; cross-checked against the xxhash package in test_golden_vectors).
HIGH_RANK_LONGS = [(555506679, 31, 13), (1608524621, 32, 27), (283986680, 33, 480),
                   (3880637358, 34, 342), (7613979340, 35, 178), (19364577309, 36, 321),
                   (56728968515, 37, 240), (379893492375, 38, 473), (483058871146, 39, 15)]


def hll_high_register_sets():
    """Register files with registers 29..56: the range where count()'s `1 << Midx` (a Scala Int
    shifted by a Long, StatefulHyperloglogPlus.scala:220) departs from 2^Midx.  Backgrounds look
    like a 1e9..1e10-distinct sketch (registers ~ 18..26) plus small / empty ones."""
    import random
    from oracle import deequ_oracle as O
    rng = random.Random(2031)
    sets = []

    def bg(center):
        return [max(1, min(30, center + int(rng.expovariate(1.0)) - int(rng.expovariate(1.0))))
                for _ in range(O.M)]
    for hi in range(29, 57):                      # one high register on a realistic background
        regs = bg(21)
        regs[rng.randrange(O.M)] = hi
        sets.append(regs)
    for k in (2, 9, 40):                          # several registers >= 31
        regs = bg(23)
        for _ in range(k):
            regs[rng.randrange(O.M)] = rng.randrange(31, 57)
        sets.append(regs)
    regs = [0] * O.M                              # linear-counting path with a 31 and a 40
    regs[3], regs[77] = 31, 40
    sets.append(regs)
    sets.append([31] * O.M)                       # zInverse < 0: negative estimate
    sets.append([32] * O.M)                       # 1 << 32 == 1 on an Int: estimate of M*M*alpha
    sets.append([31] * 256 + [1] * 256)           # zInverse == 128 - 2^-23
    return sets


def hll_high_register_vectors():
    from oracle import deequ_oracle as O
    out = []
    for regs in hll_high_register_sets():
        words = O.hll_words(regs)
        est, corrected = O.hll_count(words)
        out.append({"words": [int(w) for w in words], "estimate": est, "bias_corrected": corrected,
                    "max_register": max(regs)})
    return out


def high_rank_column_expected():
    """A 4099-row long column: 4090 values 0..4089 plus the 9 HIGH_RANK_LONGS."""
    from oracle import deequ_oracle as O
    values = list(range(4090)) + [v for v, _, _ in HIGH_RANK_LONGS]
    regs = O.hll_registers(values, "long")
    words = O.hll_words(regs)
    est, corrected = O.hll_count(words)
    return {"values_note": "range(4090) + HIGH_RANK_LONGS values", "words": [int(w) for w in words],
            "estimate": est, "bias_corrected": corrected,
            "high_rank_longs": [list(x) for x in HIGH_RANK_LONGS]}


def main():
    from oracle import deequ_oracle as O
    out = {"generator": "tests/golden/make_golden.py (oracle/deequ_oracle.py)",
           "xxh64_seed42": {}, "cases": {}}
    out["hll_high_registers"] = hll_high_register_vectors()
    out["hll_high_rank_column"] = high_rank_column_expected()
    for ty, vals in XXH_INPUTS.items():
        out["xxh64_seed42"][ty] = [[v, O.spark_xxhash64(v, ty)] for v in vals]
    for name, n, seed, null_rate, batch in CASES:
        t = golden_table(n, seed, null_rate)
        ot = oracle_table(t)
        case = {"n": n, "seed": seed, "null_rate": null_rate, "batch_rows": batch,
                "scan": {}, "freq": {}, "histogram": {}}
        for key, kind, arg, where in SCAN_AGGS:
            case["scan"][key] = scan_expected(ot, kind, arg, where)
        for cols in FREQ_COLS:
            case["freq"][",".join(cols)] = freq_expected(ot, cols)
        for col in ("c", "s"):
            case["histogram"][col] = histogram_expected(ot, col)
        out["cases"][name] = case
        print(name, "done", flush=True)
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
