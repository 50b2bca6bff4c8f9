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


def main():
    from oracle import deequ_oracle as O
    out = {"generator": "tests/golden/make_golden.py (oracle/deequ_oracle.py)",
           "xxh64_seed42": {}, "cases": {}}
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
