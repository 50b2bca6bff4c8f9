"""Evaluates a known-answer case with the ORACLE (oracle/deequ_oracle.py) -- test helper."""
import math

from oracle import deequ_oracle as O

EMPTY, FAILURE = "EMPTY", "FAILURE"
NUMERIC = O.NUM_TYPES


def oracle_metric(t: "O.OTable", cls: str, args, kwargs):
    where = kwargs.get("where")
    need_cols = []
    if cls in ("Completeness", "Sum", "Mean", "Minimum", "Maximum", "StandardDeviation",
               "ApproxCountDistinct", "Entropy"):
        need_cols = [args[0]]
    elif cls in ("Uniqueness", "Distinctness", "CountDistinct", "UniqueValueRatio"):
        need_cols = args[0] if isinstance(args[0], list) else [args[0]]
    elif cls == "Correlation":
        need_cols = [args[0], args[1]]
    for c in need_cols:
        if c not in t.columns:
            return FAILURE
    if cls in ("Sum", "Mean", "Minimum", "Maximum", "StandardDeviation", "Correlation"):
        for c in need_cols:
            if t.types[c] not in NUMERIC and not O.decimal_ps(t.types[c]):
                return FAILURE
    try:
        if cls == "Size":
            v = O.agg_conditional_count(t, where)
            return EMPTY if v is None else float(v)
        if cls == "Completeness":
            num = O.agg_sum_notnull(t, args[0], where)
            den = O.agg_conditional_count(t, where)
            if num is None or den is None:
                return EMPTY
            return float("nan") if den == 0 else num / den
        if cls == "Compliance":
            num = O.agg_compliance(t, args[1], where)
            den = O.agg_conditional_count(t, where)
            if num is None or den is None:
                return EMPTY
            return float("nan") if den == 0 else num / den
        if cls == "Sum":
            v = O.agg_sum(t, args[0], where)
            return EMPTY if v is None else v
        if cls == "Mean":
            v = O.agg_sum(t, args[0], where)
            return EMPTY if v is None else v / t.n
        if cls == "Minimum":
            v = O.agg_min(t, args[0], where)
            return EMPTY if v is None else v
        if cls == "Maximum":
            v = O.agg_max(t, args[0], where)
            return EMPTY if v is None else v
        if cls == "StandardDeviation":
            n, avg, m2 = O.agg_stddev(t, args[0], where)
            return EMPTY if n == 0 else math.sqrt(m2 / n)
        if cls == "Correlation":
            n, xa, ya, ck, xm, ym = O.agg_corr(t, args[0], args[1], where)
            if n == 0:
                return EMPTY
            den = math.sqrt(xm * ym)
            return float("nan") if den == 0 else ck / den
        if cls == "ApproxCountDistinct":
            return O.hll_count(O.agg_hll(t, args[0], where))[0]
        freq = O.frequencies(t, need_cols)
        if cls == "Uniqueness":
            v = O.uniqueness(freq, t.n)
        elif cls == "Distinctness":
            v = O.distinctness(freq, t.n)
        elif cls == "UniqueValueRatio":
            v = O.unique_value_ratio(freq)
        elif cls == "CountDistinct":
            v = O.count_distinct(freq)
        elif cls == "Entropy":
            v = O.entropy(freq, t.n)
        else:
            raise ValueError(cls)
        return EMPTY if v is None else v
    except KeyError:
        return FAILURE


def matches(got, expected, rel=1e-12):
    if isinstance(expected, str):
        if expected == "NaN":
            return isinstance(got, float) and math.isnan(got)
        return got == expected
    if isinstance(got, str):
        return False
    if math.isnan(expected):
        return math.isnan(got)
    return got == expected or abs(got - expected) <= rel * max(abs(expected), 1e-300)
