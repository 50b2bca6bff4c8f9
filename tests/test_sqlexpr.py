"""Host-side SQL predicate compiler: the forms Check emits, Spark 2.2 coercion, errors."""
import pytest

from deequ_amd import _native as N
from deequ_amd.sqlexpr import SqlError, compile_expr, parse
from deequ_amd.table import StructField, StructType

SCHEMA = StructType([StructField("item", N.UTF8), StructField("att1", N.INT32),
                     StructField("price", N.FLOAT64), StructField("flag", N.BOOL)])


def comp(sql):
    return compile_expr(sql, SCHEMA, lambda n: SCHEMA.index(n)).words


def test_is_non_negative_form():
    assert comp("att1 >= 0") == [N.X_GE, N.X_COL, 1, N.X_I64, 0]


def test_contained_in_form_with_doubled_quotes():
    w = comp("item IS NULL OR item IN ('a''b','c')")
    assert w[0] == N.X_OR and w[1] == N.X_IS_NULL and w[4] == N.X_IN and w[5] == 2


def test_range_form_double_literals():
    w = comp("price IS NULL OR (price >= 1.0 AND price <= 3.5E2)")
    assert N.X_F64 in w


def test_string_vs_number_casts_string_to_double():
    w = comp("item < 4")
    assert w[:2] == [N.X_LT, N.X_CAST_F64]
    assert w[-2] == N.X_F64  # the int literal is promoted too


def test_case_insensitive_columns():
    assert comp("ATT1 > 3") == comp("att1 > 3")


def test_between_and_not_in():
    assert comp("att1 BETWEEN 1 AND 3")[0] == N.X_AND
    assert comp("item NOT IN ('x')")[0] == N.X_NOT


@pytest.mark.parametrize("bad", ["att1 >", "nosuch > 3", "upper(item) = 'A'", "att1 > 'a' AND",
                                 "(att1 > 3"])
def test_errors(bad):
    with pytest.raises(Exception):
        comp(bad)


def test_parse_tree_shapes():
    n = parse("a > 1 AND NOT b IS NULL OR c = 'x'")
    assert n.op == "or" and n.kids[0].op == "and"


def test_cast_as_float_and_double_opcodes():
    """CAST AS FLOAT is its own opcode (rounds to float, prints as Float.toString); CAST AS DOUBLE
    widens (prints as Double.toString); a string cast to FLOAT is refused (Float.parseFloat's one
    rounding is not restated)."""
    assert comp("CAST(price AS FLOAT) > 1.5")[:2] == [N.X_GT, N.X_CAST_F32]
    assert comp("CAST(att1 AS DOUBLE) > 1.5")[:2] == [N.X_GT, N.X_CAST_F64]
    with pytest.raises(SqlError):
        comp("CAST(item AS FLOAT) > 1.5")
