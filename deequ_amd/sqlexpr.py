"""Spark-SQL predicate subset -> engine expression words (include/deequ_amd.h, dq_xop).

deequ passes SQL strings to Spark's ``expr()`` for ``where`` filters and constraints
(``Analyzers.conditionalSelection`` / ``conditionalCount``, Analyzer.scala:385-408; Compliance
Compliance.scala:47-49).  The strings Check generates are (Check.scala):

  * ``satisfies``            any predicate                                           :538-548
  * ``isNonNegative``        ``"c >= 0"``,  ``isPositive`` ``"c > 0"``               :670-686
  * ``isLessThan`` & co.     ``"a < b"``, ``"a <= b"``, ``"a > b"``, ``"a >= b"``    :697-760
  * ``isContainedIn``        ``"c IS NULL OR c IN ('v1','v2')"`` (quotes doubled)    :826-840
  * numeric range            ``"c IS NULL OR (c >= lo AND c <= hi)"``                :853-869

This module parses that grammar (plus NOT, parentheses, <>, !=, <=>, BETWEEN, booleans, NULL and
CAST(x AS DOUBLE)) and applies Spark 2.2's type coercion so the engine only sees typed operations:

  * numeric vs numeric: compared in the wider type (integral -> int64, else double);
  * string vs numeric: the string side is CAST to DOUBLE (Spark 2.2 ``PromoteStrings``);
  * ``x IN (...)`` with mixed item types: numeric literals in a string list become strings
    (``InConversion`` -> ``findWiderCommonType`` with string promotion).

Column names resolve case-insensitively (spark.sql.caseSensitive=false).  Anything outside the
grammar raises :class:`SqlError`, which the runner turns into a failure of the shared scan exactly
like Spark's AnalysisException at ``data.agg`` (AnalysisRunner.scala:310-313).
"""
from __future__ import annotations

import re
import struct
from dataclasses import dataclass, field
from typing import List, Optional

from . import _native as N


class SqlError(Exception):
    pass


# ------------------------------------------------------------------------------------------------
# Tokenizer
# ------------------------------------------------------------------------------------------------
_TOKEN = re.compile(r"""
    \s*(?:
      (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[LDSYlfdsyBD]{0,2})|
      (?P<str>'(?:[^'\\]|''|\\.)*'|"(?:[^"\\]|\\.)*")|
      (?P<bq>`(?:[^`]|``)+`)|
      (?P<op><=>|<=|>=|<>|!=|==|=|<|>|\(|\)|,|\+|-|\*|/)|
      (?P<id>[A-Za-z_][A-Za-z0-9_.]*)
    )""", re.VERBOSE)


@dataclass
class Tok:
    kind: str
    text: str


def tokenize(s: str) -> List[Tok]:
    out, pos = [], 0
    s = s.rstrip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise SqlError(f"cannot parse SQL expression at: {s[pos:]!r}")
        pos = m.end()
        for k in ("num", "str", "bq", "op", "id"):
            if m.group(k) is not None:
                out.append(Tok(k, m.group(k)))
                break
    return out


# ------------------------------------------------------------------------------------------------
# AST
# ------------------------------------------------------------------------------------------------
@dataclass
class Node:
    op: str                      # col, lit, isnull, isnotnull, not, and, or, cmp, in, cast
    kids: List["Node"] = field(default_factory=list)
    name: Optional[str] = None   # column name / comparison symbol / cast type
    value: object = None         # literal value
    ltype: Optional[str] = None  # literal type: int, float, str, bool, null
    # numeric literals: the exact value (int or decimal.Decimal) and whether Spark 2.2 types it
    # DoubleType (a D suffix; every other fractional / exponent literal is a DecimalType literal)
    exact: object = None
    dbl: bool = False


_KW = {"AND", "OR", "NOT", "IS", "NULL", "IN", "TRUE", "FALSE", "BETWEEN", "CAST", "AS", "RLIKE"}

# The engine's spelling of PatternMatch's counted expression,
# when(regexp_extract(x, pattern, 0) != "", 1).otherwise(0) (PatternMatch.scala:44-46): TRUE when
# Java's first find() match exists and is non-empty, FALSE otherwise (a NULL x included).
FIND_NONEMPTY = "dq_find_nonempty"


class _Parser:
    def __init__(self, toks: List[Tok]):
        self.t = toks
        self.i = 0

    def peek(self, k=0) -> Optional[Tok]:
        j = self.i + k
        return self.t[j] if j < len(self.t) else None

    def kw(self, word: str, k=0) -> bool:
        t = self.peek(k)
        return t is not None and t.kind == "id" and t.text.upper() == word

    def sym(self, s: str) -> bool:
        t = self.peek()
        return t is not None and t.kind == "op" and t.text == s

    def take(self) -> Tok:
        t = self.peek()
        if t is None:
            raise SqlError("unexpected end of expression")
        self.i += 1
        return t

    def expect_sym(self, s: str):
        if not self.sym(s):
            raise SqlError(f"expected '{s}'")
        self.i += 1

    def parse(self) -> Node:
        n = self.or_()
        if self.peek() is not None:
            raise SqlError(f"unexpected token {self.peek().text!r}")
        return n

    def or_(self) -> Node:
        n = self.and_()
        while self.kw("OR"):
            self.i += 1
            n = Node("or", [n, self.and_()])
        return n

    def and_(self) -> Node:
        n = self.not_()
        while self.kw("AND"):
            self.i += 1
            n = Node("and", [n, self.not_()])
        return n

    def not_(self) -> Node:
        if self.kw("NOT"):
            self.i += 1
            return Node("not", [self.not_()])
        return self.predicate()

    def predicate(self) -> Node:
        left = self.primary()
        t = self.peek()
        if t is None:
            return left
        if t.kind == "op" and t.text in ("=", "==", "<>", "!=", "<", "<=", ">", ">=", "<=>"):
            self.i += 1
            sym = {"==": "=", "!=": "<>"}.get(t.text, t.text)
            return Node("cmp", [left, self.primary()], name=sym)
        if self.kw("IS"):
            self.i += 1
            neg = False
            if self.kw("NOT"):
                self.i += 1
                neg = True
            if not self.kw("NULL"):
                raise SqlError("expected NULL after IS")
            self.i += 1
            return Node("isnotnull" if neg else "isnull", [left])
        neg = False
        if self.kw("NOT") and self.kw("RLIKE", 1):
            self.i += 1
            neg = True
        if self.kw("RLIKE"):  # x RLIKE 'java regex': find() anywhere, NULL on NULL
            self.i += 1
            pat = self.primary()
            if pat.op != "lit" or pat.ltype != "str":
                raise SqlError("RLIKE needs a string literal pattern")
            n = Node("regex", [left], name="rlike", value=pat.value)
            return Node("not", [n]) if neg else n
        if self.kw("NOT") and (self.kw("IN", 1) or self.kw("BETWEEN", 1)):
            self.i += 1
            neg = True
        if self.kw("IN"):
            self.i += 1
            self.expect_sym("(")
            items = [self.primary()]
            while self.sym(","):
                self.i += 1
                items.append(self.primary())
            self.expect_sym(")")
            n = Node("in", [left] + items)
            return Node("not", [n]) if neg else n
        if self.kw("BETWEEN"):
            self.i += 1
            lo = self.primary()
            if not self.kw("AND"):
                raise SqlError("expected AND in BETWEEN")
            self.i += 1
            hi = self.primary()
            n = Node("and", [Node("cmp", [left, lo], name=">="), Node("cmp", [left, hi], name="<=")])
            return Node("not", [n]) if neg else n
        return left

    def primary(self) -> Node:
        t = self.take()
        if t.kind == "op" and t.text == "(":
            n = self.or_()
            self.expect_sym(")")
            return n
        if t.kind == "op" and t.text in ("-", "+"):
            inner = self.primary()
            if inner.op != "lit" or inner.ltype not in ("int", "float"):
                raise SqlError("unary minus only supported on numeric literals")
            if t.text == "-":
                inner.value = -inner.value
                inner.exact = -inner.exact if inner.exact is not None else None
            return inner
        if t.kind == "num":
            return _num_literal(t.text)
        if t.kind == "str":
            q = t.text[0]
            body = t.text[1:-1]
            body = body.replace("''", "'") if q == "'" else body
            body = re.sub(r"\\(.)", lambda m: {"n": "\n", "t": "\t", "0": "\0"}.get(m.group(1), m.group(1)), body)
            return Node("lit", value=body, ltype="str")
        if t.kind == "bq":
            return Node("col", name=t.text[1:-1].replace("``", "`"))
        if t.kind == "id":
            u = t.text.upper()
            if u == "NULL":
                return Node("lit", value=None, ltype="null")
            if u in ("TRUE", "FALSE"):
                return Node("lit", value=(u == "TRUE"), ltype="bool")
            if u == "CAST":
                self.expect_sym("(")
                inner = self.or_()
                if not self.kw("AS"):
                    raise SqlError("expected AS in CAST")
                self.i += 1
                ty = self.take().text.upper()
                self.expect_sym(")")
                return Node("cast", [inner], name=ty)
            if u in _KW:
                raise SqlError(f"unexpected keyword {t.text}")
            if self.sym("(") and t.text.lower() == FIND_NONEMPTY:
                self.expect_sym("(")
                x = self.or_()
                self.expect_sym(",")
                pat = self.primary()
                self.expect_sym(")")
                if pat.op != "lit" or pat.ltype != "str":
                    raise SqlError(f"{FIND_NONEMPTY} needs a string literal pattern")
                return Node("regex", [x], name="nonempty", value=pat.value)
            if self.sym("("):
                raise SqlError(f"function {t.text}() is not supported by the engine")
            return Node("col", name=t.text)
        raise SqlError(f"unexpected token {t.text!r}")


def _num_literal(text: str) -> Node:
    m = re.match(r"^((?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?)([A-Za-z]*)$", text)
    body, suffix = m.group(1), m.group(2).upper()
    if suffix in ("D", "BD") or any(c in body for c in ".eE"):
        from decimal import Decimal
        return Node("lit", value=float(body), ltype="float", exact=Decimal(body), dbl=suffix == "D")
    if suffix in ("", "L", "S", "Y"):
        return Node("lit", value=int(body), ltype="int", exact=int(body))
    raise SqlError(f"bad numeric literal {text}")


def parse(sql: str) -> Node:
    return _Parser(tokenize(sql)).parse()


# ------------------------------------------------------------------------------------------------
# Typing + emission
# ------------------------------------------------------------------------------------------------
_CMP = {"=": N.X_EQ, "<>": N.X_NE, "<": N.X_LT, "<=": N.X_LE, ">": N.X_GT, ">=": N.X_GE,
        "<=>": N.X_EQ_NULL_SAFE}


def _kind_of_type(t: int) -> str:
    if t == N.UTF8:
        return "str"
    if t == N.BOOL:
        return "bool"
    if t in N.INTEGRAL_TYPES:
        return "int"
    if N.is_decimal(t):
        return "dec"
    if t == N.DATE32:
        return "date"
    if t == N.TIMESTAMP_US:
        return "ts"
    if t == N.UNSUPPORTED:
        raise SqlError("a column of a type the engine does not read appears in an expression")
    return "float"


_DEC_LIMIT = 10 ** 38  # |unscaled| of any decimal(38) value is below it


def _dec128_words(v: int) -> List[int]:
    """An unscaled value (clamped to +-10^38: still on the right side of every column value) as
    the [X_DEC128, lo, hi] words (signed int64 each)."""
    v = max(-_DEC_LIMIT, min(_DEC_LIMIT, v)) & ((1 << 128) - 1)
    lo, hi = v & 0xFFFFFFFFFFFFFFFF, v >> 64
    sg = lambda x: x - (1 << 64) if x >= (1 << 63) else x  # noqa: E731
    return [N.X_DEC128, sg(lo), sg(hi)]


def _exact_literal(n: "Node"):
    """The exact value of an int / decimal literal (None for a double literal or a non-number)."""
    if n.op != "lit" or n.ltype not in ("int", "float") or n.dbl or n.exact is None:
        return None
    return n.exact


class _Emitter:
    def __init__(self, schema, col_index):
        self.schema = schema
        self.col_index = col_index  # callable name -> column index in the plan
        self.words: List[int] = []
        self.columns: List[str] = []

    def type_of(self, n: Node) -> str:
        if n.op == "col":
            name = self.schema.resolve(n.name)
            if name is None:
                raise SqlError(f"cannot resolve '`{n.name}`' given input columns: "
                               f"[{', '.join(self.schema.field_names)}]")
            n.name = name
            return _kind_of_type(self.schema[name].dtype)
        if n.op == "lit":
            return n.ltype
        if n.op == "cast":
            return {"DOUBLE": "float", "FLOAT": "float", "STRING": "str", "INT": "int",
                    "BIGINT": "int", "LONG": "int", "BOOLEAN": "bool"}.get(n.name, "?")
        return "bool"

    def emit(self, n: Node, want: Optional[str] = None):
        w = self.words
        if n.op == "col":
            self.type_of(n)
            w += [N.X_COL, self.col_index(n.name)]
            if n.name not in self.columns:
                self.columns.append(n.name)
            if want == "float" and self.type_of(n) in ("str", "dec"):
                w.insert(len(w) - 2, N.X_CAST_F64)  # (a decimal: Decimal.toDouble)
            return
        if n.op == "lit":
            v, t = n.value, n.ltype
            if want == "str" and t in ("int", "float"):
                v, t = (str(v) if t == "int" else repr(float(v))), "str"
            if want == "float" and t == "int":
                v, t = float(v), "float"
            if t == "null":
                w.append(N.X_NULL)
            elif t == "bool":
                w += [N.X_BOOL, 1 if v else 0]
            elif t == "int":
                if not -(1 << 63) <= v < (1 << 63):
                    raise SqlError(f"integer literal out of range: {v}")
                w += [N.X_I64, v]
            elif t == "float":
                w += [N.X_F64, struct.unpack("<q", struct.pack("<d", v))[0]]
            elif t == "str":
                b = v.encode("utf-8")
                w += [N.X_STR, len(b)]
                padded = b + b"\0" * ((-len(b)) % 8)
                w += list(struct.unpack(f"<{len(padded) // 8}q", padded)) if padded else []
            return
        if n.op == "cast":
            if n.name not in ("DOUBLE", "FLOAT"):
                raise SqlError(f"CAST AS {n.name} is not supported by the engine")
            if n.name == "FLOAT" and self.type_of(n.kids[0]) == "str":
                # Spark parses with Float.parseFloat (one rounding to float); parse-to-double and
                # then round would round twice -- refused rather than restated approximately
                raise SqlError("CAST(string AS FLOAT) is not supported by the engine")
            w.append(N.X_CAST_F32 if n.name == "FLOAT" else N.X_CAST_F64)
            self.emit(n.kids[0])
            return
        if n.op in ("isnull", "isnotnull", "not"):
            w.append({"isnull": N.X_IS_NULL, "isnotnull": N.X_IS_NOT_NULL, "not": N.X_NOT}[n.op])
            if n.op == "not" and self.type_of(n.kids[0]) not in ("bool", "null"):
                raise SqlError("NOT needs a boolean operand")
            self.emit(n.kids[0])
            return
        if n.op in ("and", "or"):
            for k in n.kids:
                if self.type_of(k) not in ("bool", "null"):
                    raise SqlError(f"{n.op.upper()} needs boolean operands")
            w.append(N.X_AND if n.op == "and" else N.X_OR)
            self.emit(n.kids[0])
            self.emit(n.kids[1])
            return
        if n.op == "cmp":
            a, b = n.kids
            ta, tb = self.type_of(a), self.type_of(b)
            if "dec" in (ta, tb) and self._emit_dec_cmp(n.name, a, ta, b, tb):
                return
            for t in (ta, tb):
                if t in ("date", "ts"):
                    raise SqlError("comparisons of date / timestamp columns are not supported by "
                                   "the engine")
            target = _common_cmp_type(ta, tb)
            w.append(_CMP[n.name])
            self.emit(a, target)
            self.emit(b, target)
            return
        if n.op == "in":
            x, items = n.kids[0], n.kids[1:]
            tx = self.type_of(x)
            tis = [self.type_of(i) for i in items]
            if tx == "dec":
                self._emit_dec_in(x, items)
                return
            if tx in ("date", "ts") or any(t in ("dec", "date", "ts") for t in tis):
                raise SqlError("IN over a date / timestamp / decimal value is not supported by the "
                               "engine")
            target = tx
            if any(t not in (tx, "null") for t in tis):
                kinds = {tx} | {t for t in tis if t != "null"}
                if "str" in kinds:
                    target = "str"
                elif kinds <= {"int", "float"}:
                    target = "float" if "float" in kinds else "int"
                else:
                    raise SqlError("incompatible types in IN list")
            w += [N.X_IN, len(items)]
            self.emit(x, target if target != tx or tx == "str" else None)
            for i in items:
                self.emit(i, target)
            return
        if n.op == "regex":
            tx = self.type_of(n.kids[0])
            # a non-string operand is matched as Spark's cast to string: decimal integers,
            # true / false, Double.toString / Float.toString (csrc/jfmt.h, on the device)
            if tx not in ("str", "int", "float", "bool", "null", "dec", "date", "ts"):
                raise SqlError(f"cannot match a regex against a {tx} value")
            blob = _compiled_regex(n.value, n.name == "rlike")
            w += [N.X_REGEX, 1 if n.name == "nonempty" else 0, len(blob)]
            padded = blob + b"\0" * ((-len(blob)) % 8)
            w += list(struct.unpack(f"<{len(padded) // 8}q", padded))
            self.emit(n.kids[0])
            return
        raise SqlError(f"unsupported expression node {n.op}")

    # -- decimal columns (Spark 2.2 DecimalPrecision: exact against integral / decimal literals,
    #    through Cast(AS DOUBLE) against doubles)
    def _scale_of(self, n: Node) -> int:
        return N.decimal_scale(self.schema[self.schema.resolve(n.name)].dtype)

    def _emit_dec_cmp(self, sym: str, a: Node, ta: str, b: Node, tb: str) -> bool:
        """Emits a comparison with a decimal column operand; False when it is not one of the forms
        handled here (the generic path then raises or casts)."""
        if ta == "dec" and tb == "dec":
            raise SqlError("comparisons of two decimal values are not supported by the engine")
        col, lit, op = (a, b, sym) if ta == "dec" else (b, a, _FLIP.get(sym, sym))
        tl = tb if ta == "dec" else ta
        if tl in ("float", "str") and _exact_literal(lit) is None:
            return False  # double / string: both sides as double (Cast(decimal AS DOUBLE))
        if tl == "null":
            self.words.append(_CMP[sym])
            self.emit(a)
            self.emit(b)
            return True
        exact = _exact_literal(lit)
        if exact is None:
            raise SqlError("a decimal column compared with a non-literal value is not supported by "
                           "the engine")
        from fractions import Fraction
        t = Fraction(exact) * 10 ** self._scale_of(col)
        if t.denominator == 1:
            op, v = op, int(t)
        elif op in ("<", "<="):  # x < t  <=>  x <= floor(t)  (x an integer)
            op, v = "<=", t.numerator // t.denominator
        elif op in (">", ">="):
            op, v = ">=", -((-t.numerator) // t.denominator)
        else:  # =, <>, <=> against a value no column value equals
            v = _DEC_LIMIT
        self.words.append(_CMP[op])
        self.emit(col)
        self.words.extend(_dec128_words(v))
        return True

    def _emit_dec_in(self, x: Node, items: List[Node]) -> None:
        from fractions import Fraction
        sc = self._scale_of(x)
        words = []
        for it in items:
            if self.type_of(it) == "null":
                words.append(N.X_NULL)
                continue
            exact = _exact_literal(it)
            if exact is None:
                raise SqlError("a decimal column IN a list of non-literal / double items is not "
                               "supported by the engine")
            t = Fraction(exact) * 10 ** sc
            words.extend(_dec128_words(int(t) if t.denominator == 1 else _DEC_LIMIT))
        self.words += [N.X_IN, len(items)]
        self.emit(x)
        self.words.extend(words)


_FLIP = {"<": ">", "<=": ">=", ">": "<", ">=": "<="}


_REGEX_CACHE = {}


def _compiled_regex(pattern: str, any_match: bool) -> bytes:
    """The automaton blob of a Java regex (deequ_amd/regex.py).  RLIKE (any_match) is find()
    including an empty match: a pattern that can match the empty string then matches every row."""
    from .regex import PatternNotSupported, accept_all, compile_java_regex, nullable_pattern
    key = (pattern, any_match)
    if key not in _REGEX_CACHE:
        try:
            if any_match and nullable_pattern(pattern):
                _REGEX_CACHE[key] = accept_all(pattern).blob()
            else:
                _REGEX_CACHE[key] = compile_java_regex(pattern).blob()
        except PatternNotSupported as e:
            raise SqlError(f"regex /{pattern}/: {e}") from e
    return _REGEX_CACHE[key]


def _common_cmp_type(ta: str, tb: str) -> Optional[str]:
    if ta == "null" or tb == "null":
        return None
    if "dec" in (ta, tb) and ({ta, tb} - {"dec"}) <= {"float", "str"}:
        return "float"  # decimal vs double (or a string cast to double): Cast(decimal AS DOUBLE)
    if ta == tb:
        return ta if ta != "int" else None
    if {ta, tb} <= {"int", "float"}:
        return "float"
    if "str" in (ta, tb) and ({ta, tb} & {"int", "float"}):
        return "float"  # Spark 2.2 PromoteStrings: string side cast to double
    if "bool" in (ta, tb):
        raise SqlError(f"cannot compare {ta} with {tb}")
    return None


@dataclass
class CompiledExpr:
    sql: str
    words: List[int]
    columns: List[str]


def compile_expr(sql: str, schema, col_index) -> CompiledExpr:
    """Parses and types ``sql`` against ``schema``; ``col_index(name)`` returns the plan column
    index of a (resolved) column name."""
    node = parse(sql)
    em = _Emitter(schema, col_index)
    t = em.type_of(node) if node.op != "col" else em.type_of(node)
    if t not in ("bool", "null") and node.op in ("col", "lit"):
        if t != "bool":
            raise SqlError(f"expression '{sql}' is not a predicate")
    em.emit(node)
    return CompiledExpr(sql, em.words, em.columns)


def referenced_columns(sql: str) -> List[str]:
    out = []

    def walk(n: Node):
        if n.op == "col" and n.name not in out:
            out.append(n.name)
        for k in n.kids:
            walk(k)

    walk(parse(sql))
    return out
