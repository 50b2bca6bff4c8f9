"""The reference's test fixtures as data (src/test/scala/com/amazon/deequ/utils/FixtureSupport.scala
and NullHandlingTests.scala:14-35), with their Spark column types."""
from decimal import Decimal

FIXTURES = {
    # FixtureSupport.scala:29-46
    "dfMissing": ({
        "item": ["1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12"],
        "att1": ["a", "b", None, "a", "a", None, None, "b", "a", None, None, None],
        "att2": ["f", "d", "f", None, "f", "d", "d", None, "f", None, "f", "d"],
    }, {"item": "string", "att1": "string", "att2": "string"}),
    # FixtureSupport.scala:48-57
    "dfFull": ({
        "item": ["1", "2", "3", "4"],
        "att1": ["a", "a", "a", "b"],
        "att2": ["c", "c", "c", "d"],
    }, {"item": "string", "att1": "string", "att2": "string"}),
    # FixtureSupport.scala:59-68
    "dfWithNegativeNumbers": ({
        "item": ["1", "2", "3", "4"],
        "att1": ["-1", "-2", "-3", "-4"],
        "att2": ["-1.0", "-2.0", "-3.0", "-4.0"],
    }, {"item": "string", "att1": "string", "att2": "string"}),
    # FixtureSupport.scala:125-136
    "dfWithNumericValues": ({
        "item": ["1", "2", "3", "4", "5", "6"],
        "att1": [1, 2, 3, 4, 5, 6],
        "att2": [0, 0, 0, 5, 6, 7],
    }, {"item": "string", "att1": "int", "att2": "int"}),
    # FixtureSupport.scala:138-148
    "dfWithNumericFractionalValues": ({
        "item": ["1", "2", "3", "4", "5", "6"],
        "att1": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0],
        "att2": [0.0, 0.0, 0.0, 5.0, 6.0, 7.0],
    }, {"item": "string", "att1": "double", "att2": "double"}),
    # FixtureSupport.scala:150-163
    "dfWithUniqueColumns": ({
        "unique": ["1", "2", "3", "4", "5", "6"],
        "nonUnique": ["0", "0", "0", "5", "6", "7"],
        "nonUniqueWithNulls": ["3", "3", "3", None, None, None],
        "uniqueWithNulls": ["1", "2", None, "3", "4", "5"],
        "onlyUniqueWithOtherNonUnique": ["5", "6", "7", "0", "0", "0"],
        "halfUniqueCombinedWithNonUnique": ["0", "0", "0", "4", "5", "6"],
    }, {k: "string" for k in ["unique", "nonUnique", "nonUniqueWithNulls", "uniqueWithNulls",
                              "onlyUniqueWithOtherNonUnique", "halfUniqueCombinedWithNonUnique"]}),
    # FixtureSupport.scala:165-176
    "dfWithDistinctValues": ({
        "att1": ["a", "a", None, "b", "b", "c"],
        "att2": [None, None, "x", "x", "x", "y"],
    }, {"att1": "string", "att2": "string"}),
    # FixtureSupport.scala:178-185
    "dfWithConditionallyUninformativeColumns": ({
        "att1": [1, 2, 3], "att2": [0, 0, 0],
    }, {"att1": "int", "att2": "int"}),
    # FixtureSupport.scala:187-194
    "dfWithConditionallyInformativeColumns": ({
        "att1": [1, 2, 3], "att2": [4, 5, 6],
    }, {"att1": "int", "att2": "int"}),
    # NullHandlingTests.scala:14-35 (two partitions in the reference)
    "dataWithNullColumns": ({
        "stringCol": [None] * 8,
        "numericCol": [None] * 8,
        "numericCol2": [None] * 8,
        "numericCol3": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0],
    }, {"stringCol": "string", "numericCol": "double", "numericCol2": "double",
        "numericCol3": "double"}),
    # AnalyzerTests.scala:508 -- sparkContext.range(-1000, 1000)
    "range2000": ({"att1": list(range(-1000, 1000))}, {"att1": "long"}),
    # AnalyzerTests.scala:454-466 -- three rows of DecimalType.SYSTEM_DEFAULT = decimal(38,18)
    # (Scala's BigDecimal(123.45) of a double is decimal("123.45"))
    "dfDecimalMinimum": ({"num": [Decimal("123.45"), Decimal("99"), Decimal("678")]},
                         {"num": "decimal(38,18)"}),
    # examples/BasicExample.scala:29-34 (Item entity, entities.scala:19-25)
    "basicExampleItems": ({
        "id": [1, 2, 3, 4, 5],
        "name": ["Thingy A", "Thingy B", None, "Thingy D", "Thingy E"],
        "description": ["awesome thing.", "available at http://thingb.com", None,
                        "checkout https://thingd.ca", None],
        "priority": ["high", None, "low", "low", "high"],
        "numViews": [0, 0, 5, 10, 12],
    }, {"id": "long", "name": "string", "description": "string", "priority": "string",
        "numViews": "long"}),
}

ARROW_TYPES = {"string": "string", "int": "int32", "long": "int64", "double": "float64",
               "float": "float32", "boolean": "bool_", "short": "int16", "byte": "int8"}


def arrow_type(ty: str):
    """The Arrow type of an oracle / Spark type name (decimal(p,s), date, timestamp included)."""
    import re

    import pyarrow as pa
    m = re.match(r"^decimal\((\d+),(\d+)\)$", ty)
    if m:
        return pa.decimal128(int(m.group(1)), int(m.group(2)))
    if ty == "date":
        return pa.date32()
    if ty == "timestamp":
        return pa.timestamp("us")
    return getattr(pa, ARROW_TYPES[ty])()


def arrow_table(name):
    import pyarrow as pa
    cols, types = FIXTURES[name]
    arrays = [pa.array(v, type=arrow_type(types[k])) for k, v in cols.items()]
    return pa.Table.from_arrays(arrays, names=list(cols))


def oracle_table(name):
    from oracle.deequ_oracle import OTable
    cols, types = FIXTURES[name]
    return OTable({k: list(v) for k, v in cols.items()}, dict(types))
