"""Java regular expressions -> byte DFAs for the device (PatternMatch, PatternMatch.scala:41-53).

PatternMatch counts a row when ``regexp_extract(col, pattern, 0) != ""``: Java's first
``Matcher.find()`` match exists and is non-empty.  For a pattern that cannot match the empty string
(every pattern of ``Patterns``, PatternMatch.scala:57-72) that is "some substring matches", a
regular property of the row's UTF-8 bytes, so the pattern compiles to ONE deterministic automaton
over bytes the device runs per row (deequ_amd/csrc/expr.hip, XI_REGEX): no backtracking, no
per-row allocation.

Language model.  The automaton reads the whole row and then an end-of-text symbol (EOT, class
256), and accepts iff the row is in  Sigma* P Sigma* EOT.  Lookaheads and word boundaries are
compiled in continuation-passing style: ``(?!X)`` at a point whose continuation (the rest of the
pattern, then Sigma* EOT) is C becomes  C minus (X Sigma* EOT), a product construction on the two
DFAs.  The DFA's states from which every input is accepted / rejected are marked so the device
stops early.

Supported Java syntax: literals and escapes (\\t \\n \\r \\f \\a \\e \\xhh \\uhhhh \\0o \\cX and
escaped metacharacters), ``.`` (any code point but the Java line terminators), classes with ranges,
negation, nested escapes and \\d \\D \\s \\S \\w \\W (ASCII, as Java without UNICODE_CHARACTER_CLASS),
\\h \\H \\v \\V \\R, the US-ASCII POSIX classes \\p{Lower} ... \\p{Space} and their \\P{...}
complements, \\Q...\\E (Pattern.java's RemoveQEQuoting, before parsing), groups ( ), (?: ),
named groups (?<name> ) with \\k<name>, class unions [a[b]] and intersections [a-z&&[^b]],
alternation, greedy / lazy quantifiers * + ? {n} {n,} {n,m}, lookaheads (?= )
(?! ), back-references to groups with a finite language (expanded: the CREDITCARD separators),
^ / \\A at the start; $ / \\Z (end, or before one final line terminator, "\\r\\n" included) and
\\z (strict end) at the end; \\b at the start or end of the pattern; anchors, \\b / \\B and
bounded lookbehinds inside the pattern (see _rewrite_inner_anchors); the embedded flags
(?idmsux-idmsux) and (?idmsux-idmsux: ) anywhere, each to the end of the enclosing group,
alternatives included: i (ASCII case folding, Java without UNICODE_CASE), d (UNIX_LINES), m
(MULTILINE: Pattern.java's Caret / Dollar(true) and their UNIX_LINES forms), s (DOTALL), x
(COMMENTS: white space and #-comments skipped wherever Java's parser peeks, classes included), u
(no effect without i).

Nullable patterns (``\\d*``, ``(?i)x?y*``, ``[0-9]*(\\.[0-9]+)?``): the empty match at offset 0
always exists, so find()'s first match starts there and the row counts iff Java's PREFERRED
match at offset 0 is non-empty -- compiled from a priority-ordered thread automaton
(``compile_nullable``: alternation order, greedy / lazy preference, Java's rule that an iteration
consuming nothing ends its loop), with no anchor but a leading ^.

A lookahead inside a quantifier (``a(?:(?!b).)*c``, the "tempered dot") cannot be compiled
against its continuation, which loops back through it: it becomes an obligation instead -- a
thread of the subset construction that crosses it carries the lookahead's automaton, advanced
with every symbol, and dies when it fails (_determinize_obligations).

Rejected (a PatternNotSupported error, never a silently different answer): nullable patterns with
a lookaround, back-reference or trailing anchor, possessive quantifiers over more than one
character class (over one, C*+ is C*(?!C)), atomic groups over unbounded languages (see
_Parser._atomic), unbounded lookbehinds,
the flags U and i with u, anchors / lookbehinds the automaton cannot place (after a lookahead, or
inside a lookaround), $ after a pattern that may end in "\\r" (Java's $ never matches between
"\\r\\n"), and automata above ``MAX_STATES``.

\\b is Java's Bound: a word character is '_' or Character.isLetterOrDigit (categories L* and Nd),
taken from Python's Unicode database.  Exact for U+0000-U+07FF and the punctuation / symbol blocks
U+2000-U+2BFF, U+3000-U+303F, U+FF00-U+FFEF (the em dash and the euro sign are boundaries, as in
Java); other code points from U+0800 up count as word characters (overwhelmingly letters: CJK,
Indic, Hangul ...), which keeps the byte automaton small.  Parity unpinned: those other blocks,
JDK 8's Unicode 6.2 tables vs Python's, and Java's rule that a combining mark (Mn) after a base
character is a word character.
"""
from __future__ import annotations

import functools
import unicodedata

import struct
from dataclasses import dataclass
from typing import Dict, FrozenSet, List, Optional, Sequence, Tuple

EOT = 256
NSYM = 257
MAX_STATES = 4096
MAX_CP = 0x10FFFF


class PatternNotSupported(ValueError):
    pass


class _NeedsObligations(PatternNotSupported):
    """Refused by the lookahead product construction only: compile_java_regex retries with every
    lookahead as an obligation (exact $, lookbehinds and ^ after lookaheads)."""


# ------------------------------------------------------------------------------------------------
# Character sets: sorted disjoint code point intervals
# ------------------------------------------------------------------------------------------------
def cs_norm(r: Sequence[Tuple[int, int]]) -> Tuple[Tuple[int, int], ...]:
    out: List[List[int]] = []
    for a, b in sorted(r):
        if out and a <= out[-1][1] + 1:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return tuple((a, b) for a, b in out)


def cs_and(a, b) -> Tuple[Tuple[int, int], ...]:
    return cs_neg(list(cs_neg(a)) + list(cs_neg(b)))


def cs_neg(r) -> Tuple[Tuple[int, int], ...]:
    out, lo = [], 0
    for a, b in cs_norm(r):
        if a > lo:
            out.append((lo, a - 1))
        lo = b + 1
    if lo <= MAX_CP:
        out.append((lo, MAX_CP))
    return tuple(out)


DIGIT = ((48, 57),)
WORD = cs_norm([(48, 57), (65, 90), (95, 95), (97, 122)])
SPACE = cs_norm([(9, 13), (32, 32)])  # [ \t\n\x0B\f\r]
LINE_TERMINATORS = cs_norm([(10, 10), (13, 13), (0x85, 0x85), (0x2028, 0x2029)])
DOT = cs_neg(LINE_TERMINATORS)
DOT_UNIX = cs_neg(((10, 10),))  # . under UNIX_LINES
# \h and \v (Pattern.java, JDK 8: horizontal / vertical white space)
HSPACE = cs_norm([(9, 9), (32, 32), (0xA0, 0xA0), (0x1680, 0x1680), (0x180E, 0x180E),
                  (0x2000, 0x200A), (0x202F, 0x202F), (0x205F, 0x205F), (0x3000, 0x3000)])
VSPACE = cs_norm([(10, 13), (0x85, 0x85), (0x2028, 0x2029)])
# \p{...}: the POSIX classes, US-ASCII only (Java without UNICODE_CHARACTER_CLASS)
_PUNCT = ((33, 47), (58, 64), (91, 96), (123, 126))
POSIX_CLASSES = {
    "Lower": ((97, 122),), "Upper": ((65, 90),), "ASCII": ((0, 127),),
    "Alpha": ((65, 90), (97, 122)), "Digit": DIGIT, "Alnum": ((48, 57), (65, 90), (97, 122)),
    "Punct": _PUNCT, "Graph": ((33, 126),), "Print": ((32, 126),), "Blank": ((9, 9), (32, 32)),
    "Cntrl": ((0, 31), (127, 127)), "XDigit": ((48, 57), (65, 70), (97, 102)),
    "Space": ((9, 13), (32, 32)),
}
ANY = ((0, MAX_CP),)
# \b's word characters are decided exactly in these blocks (see the module docstring)
_BOUND_EXACT = ((0, 0x7FF), (0x2000, 0x2BFF), (0x3000, 0x303F), (0xFF00, 0xFFEF))


@functools.lru_cache(maxsize=1)
def bound_word_chars() -> Tuple[Tuple[int, int], ...]:
    """Java's Bound.isWord: '_' or Character.isLetterOrDigit, exact in _BOUND_EXACT, and every
    other code point from U+0800 up counted as a word character."""
    out, start = [], None
    for cp in range(MAX_CP + 1):
        if any(a <= cp <= b for a, b in _BOUND_EXACT):
            cat = unicodedata.category(chr(cp))
            w = cp == 95 or cat[0] == "L" or cat == "Nd"
        else:
            w = cp >= 0x800 and not 0xD800 <= cp <= 0xDFFF
        if w and start is None:
            start = cp
        elif not w and start is not None:
            out.append((start, cp - 1))
            start = None
    if start is not None:
        out.append((start, MAX_CP))
    return cs_norm(out)


# ------------------------------------------------------------------------------------------------
# AST
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Chars:
    ranges: Tuple[Tuple[int, int], ...]


@dataclass(frozen=True)
class Seq:
    items: Tuple


@dataclass(frozen=True)
class Alt:
    options: Tuple


@dataclass(frozen=True)
class Repeat:
    node: object
    lo: int
    hi: Optional[int]  # None = unbounded
    greedy: bool = True  # (lazy *? +? ?? {n,m}?: the same language, another match preference)


@dataclass(frozen=True)
class Group:
    node: object
    index: Optional[int]  # capturing group number, None for (?: )


@dataclass(frozen=True)
class Look:
    node: object
    negative: bool


@dataclass(frozen=True)
class Behind:
    """(?<=X) / (?<!X): the text before the position (from the text's start) ends / does not end
    with a string of X (X of bounded length, as Java requires)."""
    node: object
    negative: bool


@dataclass(frozen=True)
class BackRef:
    index: int


@dataclass(frozen=True)
class Anchor:
    kind: str  # "^", "$", "\\b"


@dataclass(frozen=True)
class DollarLook(Look):
    """Java's $ inside a pattern, as the lookahead (?=(\\r\\n|[line terminator])?END)."""


@dataclass(frozen=True)
class EndText:
    """Inside a lookahead only: the text ends here (the anchors inside a pattern, see
    _rewrite_inner_anchors)."""


EMPTY = Seq(())


def _remove_qe_quoting(p: str) -> str:
    """\\Q...\\E as Pattern.java's RemoveQEQuoting does it, before parsing: each quoted ASCII
    character that is not a letter or digit is escaped (so a following quantifier binds to the
    last quoted character, and classes see literals); an unterminated \\Q runs to the end."""
    out, i, n = [], 0, len(p)
    while i < n:
        if p[i] == "\\" and i + 1 < n and p[i + 1] == "Q":
            j = p.find("\\E", i + 2)
            j = n if j < 0 else j
            for k, ch in enumerate(p[i + 2:j]):
                if ch.isascii() and ch.isdigit() and k == 0:
                    # a digit first in the section becomes \x3N, so an octal escape or a
                    # back-reference just before the \Q cannot absorb it (RemoveQEQuoting's
                    # beginQuote)
                    out.append("\\x3" + ch)
                else:
                    out.append(ch if not ch.isascii() or ch.isalnum() else "\\" + ch)
            i = j + 2
        elif p[i] == "\\":
            out.append(p[i:i + 2])
            i += 2
        else:
            out.append(p[i])
            i += 1
    return "".join(out)


def _preference_order(n, cap: int):
    """The sequences of character classes X can match, in Java's backtracking order (alternatives
    left to right, a greedy repeat's next iteration before its exit), or None when X has
    anything else (an unbounded repeat, a lookaround, a nullable repeated body) or more than
    `cap` of them."""
    if isinstance(n, Chars):
        return [(n,)]
    if isinstance(n, Group):
        return _preference_order(n.node, cap)
    if isinstance(n, Seq):
        out = [()]
        for item in n.items:
            opts = _preference_order(item, cap)
            if opts is None:
                return None
            out = [a + b for a in out for b in opts]
            if len(out) > cap:
                return None
        return out
    if isinstance(n, Alt):
        out = []
        for o in n.options:
            opts = _preference_order(o, cap)
            if opts is None:
                return None
            out += opts
        return out if len(out) <= cap else None
    if isinstance(n, Repeat):
        body = _preference_order(n.node, cap)
        if n.hi is None or body is None or any(not b for b in body):
            return None

        def rep(k):
            res = []
            more = [b + r for b in body for r in rep(k + 1)] if k < n.hi else []
            stop = [()] if k >= n.lo else []
            res = more + stop if n.greedy else stop + more
            if len(res) > cap:
                raise OverflowError
            return res
        try:
            return rep(0)
        except OverflowError:
            return None
    return None


class _Parser:
    # Java's embedded flags, each to the end of its group (or inside a (?flags:...) group)
    FLAGS = ("ci", "unix", "multiline", "dotall", "ucase", "comments")
    FLAG_LETTERS = {"i": "ci", "d": "unix", "m": "multiline", "s": "dotall", "u": "ucase",
                    "x": "comments"}

    def __init__(self, pattern: str):
        self.s = _remove_qe_quoting(pattern)
        self.i = 0
        self.groups = 0
        self.names: Dict[str, int] = {}
        self.ci = False  # CASE_INSENSITIVE ((?i)): ASCII letters only, as Java without UNICODE_CASE
        self.unix = False  # UNIX_LINES ((?d)): '\n' is the only line terminator of . ^ $
        self.multiline = False  # MULTILINE ((?m)): ^ / $ at line starts / ends too
        self.dotall = False  # DOTALL ((?s)): . matches line terminators too
        self.ucase = False  # UNICODE_CASE ((?u)): refused together with (?i)
        self.comments = False  # COMMENTS ((?x)): white space and #-comments in the pattern ignored

    def _flags(self):
        return tuple(getattr(self, f) for f in self.FLAGS)

    def _set_flags(self, v):
        for f, x in zip(self.FLAGS, v):
            setattr(self, f, x)

    def _skip_comments(self):
        """COMMENTS mode: Java's peekPastWhitespace -- ASCII white space, and '#' up to the end of
        the line (UNIX_LINES: '\n'), are skipped wherever the parser peeks or takes a
        character, inside classes too, but never right after a backslash."""
        while self.i < len(self.s):
            c = self.s[self.i]
            if c in " \t\n\x0b\f\r":
                self.i += 1
            elif c == "#":
                while self.i < len(self.s):
                    c = self.s[self.i]
                    self.i += 1
                    if c == "\n" or (not self.unix and c in "\r\x85\u2028\u2029"):
                        break
            else:
                break

    def error(self, msg):
        raise PatternNotSupported(f"{msg} at position {self.i} of /{self.s}/")

    def peek(self):
        if self.comments:
            self._skip_comments()
        return self.s[self.i] if self.i < len(self.s) else None

    def take(self):
        if self.comments:
            self._skip_comments()
        return self.take_raw()

    def take_raw(self):
        c = self.s[self.i]
        self.i += 1
        return c

    def parse(self):
        node = self.alt()
        if self.i != len(self.s):
            self.error("unbalanced ')'")
        return node

    def alt(self):
        opts = [self.seq()]
        while self.peek() == "|":
            self.take()
            opts.append(self.seq())
        return opts[0] if len(opts) == 1 else Alt(tuple(opts))

    def seq(self):
        items = []
        while self.peek() is not None and self.peek() not in "|)":
            node = self.quantified()
            if node is not EMPTY:  # (an inline flag)
                items.append(node)
        return items[0] if len(items) == 1 else Seq(tuple(items))

    def quantified(self):
        atom = self.atom()
        while True:
            c = self.peek()
            if c == "*":
                self.take()
                lo, hi = 0, None
            elif c == "+":
                self.take()
                lo, hi = 1, None
            elif c == "?":
                self.take()
                lo, hi = 0, 1
            elif c == "{" and self._is_counted():
                lo, hi = self._counted()
            else:
                return atom
            if isinstance(atom, (Anchor, Look)):
                self.error("quantified assertion")
            greedy = True
            if self.peek() == "?":  # lazy: the same language, shortest first
                self.take()
                greedy = False
            elif self.peek() == "+":  # possessive: C*+ never gives back a C
                self.take()
                atom = self._possessive(atom, lo, hi)
                continue
            atom = Repeat(atom, lo, hi, greedy)

    def _possessive(self, atom, lo, hi):
        """C{lo,hi}+ over one character class C: as many C as there are, up to hi, never fewer --
        C{lo,}(?!C), or C{hi} | C{lo,hi-1}(?!C).  (Over anything longer the committed match is
        not a regular property of the text here.)"""
        if not isinstance(atom, Chars):
            self.error("possessive quantifier over more than one character class")
        if hi is not None and hi == lo:
            return Repeat(atom, lo, hi, True)
        stop = Look(atom, True)
        if hi is None:
            return Seq((Repeat(atom, lo, None, True), stop))
        return Alt((Repeat(atom, hi, hi, True), Seq((Repeat(atom, lo, hi - 1, True), stop))))

    def _atomic(self, x):
        """(?>X): the first match of X in backtracking order, never given back.  One character
        class repeated is the possessive form; a finite X is the alternation, over X's sequences
        s1, s2, ... in that order, of "s_k where no earlier s_j starts here"."""
        while isinstance(x, Group):
            x = x.node
        if isinstance(x, Repeat) and isinstance(x.node, Chars):
            return self._possessive(x.node, x.lo, x.hi) if x.greedy else Repeat(x.node, x.lo, x.lo, True)
        seqs = _preference_order(x, 32)
        if seqs is None:
            self.error("atomic group over an unbounded or large language")
        opts = []
        for k, sk in enumerate(seqs):
            if any(seqs[j] == sk for j in range(k)):
                continue
            opts.append(Seq(tuple(Look(Seq(seqs[j]), True) for j in range(k)) + sk))
        return Alt(tuple(opts)) if len(opts) != 1 else opts[0]

    def _is_counted(self):
        j = self.i + 1
        while j < len(self.s) and (self.s[j].isdigit() or self.s[j] == ","):
            j += 1
        return j < len(self.s) and self.s[j] == "}" and j > self.i + 1 and self.s[self.i + 1].isdigit()

    def _counted(self):
        self.take()
        j = self.s.index("}", self.i)
        body = self.s[self.i:j]
        self.i = j + 1
        if "," in body:
            a, b = body.split(",", 1)
            return int(a), (int(b) if b else None)
        return int(body), int(body)

    def _group_body(self):
        """A group's alternatives; an inline flag inside applies up to the group's end."""
        saved = self._flags()
        node = self.alt()
        self._set_flags(saved)
        return node

    def atom(self):
        c = self.take()
        if c == "(":
            flags = self._inline_flags()
            if flags is not None:  # (?imsx-imsx): up to the end of the enclosing group
                new, scoped = flags
                if not scoped:
                    self._set_flags(new)
                    return EMPTY
                saved = self._flags()
                self._set_flags(new)
                node = Group(self._group_body(), None)
                self._set_flags(saved)
            elif self.s.startswith("?:", self.i):
                self.i += 2
                node = Group(self._group_body(), None)
            elif self.s.startswith("?!", self.i) or self.s.startswith("?=", self.i):
                neg = self.s[self.i + 1] == "!"
                self.i += 2
                node = Look(self.alt(), neg)
            elif self.s.startswith("?<=", self.i) or self.s.startswith("?<!", self.i):
                neg = self.s[self.i + 2] == "!"
                self.i += 3
                node = Behind(self.alt(), neg)
            elif self.s.startswith("?>", self.i):  # (?>X): atomic
                self.i += 2
                node = self._atomic(self._group_body())
            elif self.s.startswith("?<", self.i):  # (?<name>X): a capturing group with a name
                j = self.s.find(">", self.i)
                name = self.s[self.i + 2:j] if j > 0 else ""
                if not (name[:1].isascii() and name[:1].isalpha() and name.isascii()
                        and name.isalnum()):
                    self.error("bad group name")
                if name in self.names:
                    self.error(f"named group <{name}> defined twice")
                self.i = j + 1
                self.groups += 1
                self.names[name] = idx = self.groups
                node = Group(self._group_body(), idx)
            elif self.peek() == "?":
                self.error("unsupported group construct (named group, atomic group or flag)")
            else:
                self.groups += 1
                idx = self.groups
                node = Group(self._group_body(), idx)
            if self.peek() != ")":
                self.error("missing ')'")
            self.take()
            return node
        if c == "[":
            return Chars(self.char_class())
        if c == ".":
            return Chars(ANY if self.dotall else DOT_UNIX if self.unix else DOT)
        if c == "^":
            return Anchor("^" + ("m" if self.multiline else "") + ("d" if self.multiline and self.unix else ""))
        if c == "$":
            return Anchor("$" + ("m" if self.multiline else "") + ("d" if self.unix else ""))
        if c == "\\":
            return self.escape(in_class=False)
        if c in "*+?":
            self.error("dangling quantifier")
        return Chars(self.fold(((ord(c), ord(c)),)))

    def _inline_flags(self):
        """At '(' : (?flags-flags) -> (the new flag tuple, False); (?flags-flags: -> (the
        group's flag tuple, True), consumed; else None.  Flags: i d m s u x; U
        (UNICODE_CHARACTER_CLASS) is refused, and so is u together with i (Unicode case
        folding)."""
        j = self.i
        if not (self.s.startswith("?", j) and j + 1 < len(self.s)
                and (self.s[j + 1].isalpha() or self.s[j + 1] == "-")):
            return None
        j += 1
        vals = dict(zip(self.FLAGS, self._flags()))
        on = True
        while j < len(self.s) and self.s[j] not in "):":
            c = self.s[j]
            if c == "-" and on:
                on = False
            elif c in self.FLAG_LETTERS:
                vals[self.FLAG_LETTERS[c]] = on
            elif c == "U":
                self.i = j
                self.error("the UNICODE_CHARACTER_CLASS flag (?U)")
            else:
                self.i = j
                self.error(f"unknown inline flag {c!r}")
            j += 1
        if j >= len(self.s):
            self.error("unterminated inline flag group")
        self.i = j + 1
        return tuple(vals[f] for f in self.FLAGS), self.s[j] == ":"

    def fold(self, ranges):
        """Under (?i): the ranges plus the other case of every ASCII letter in them."""
        if not self.ci:
            return ranges
        if self.ucase:
            self.error("case-insensitive matching with UNICODE_CASE (?iu)")
        extra = []
        for a, b in ranges:
            for lo, hi, d in ((65, 90, 32), (97, 122, -32)):
                x, y = max(a, lo), min(b, hi)
                if x <= y:
                    extra.append((x + d, y + d))
        return cs_norm(list(ranges) + extra)

    def escape(self, in_class: bool):
        if self.i >= len(self.s):  # (raw: COMMENTS mode skips nothing after a backslash)
            self.error("trailing backslash")
        c = self.take_raw()
        simple = {"t": 9, "n": 10, "r": 13, "f": 12, "a": 7, "e": 27}
        if c in simple:
            v = simple[c]
            return Chars(((v, v),)) if not in_class else ((v, v),)
        classes = {"d": DIGIT, "D": cs_neg(DIGIT), "s": SPACE, "S": cs_neg(SPACE), "w": WORD,
                   "W": cs_neg(WORD), "h": HSPACE, "H": cs_neg(HSPACE), "v": VSPACE,
                   "V": cs_neg(VSPACE)}
        if c in classes:
            return Chars(classes[c]) if not in_class else classes[c]
        if c in "pP":  # \p{Name} / \pL: the POSIX classes only
            if self.s.startswith("{", self.i):
                j = self.s.find("}", self.i)
                if j < 0:
                    self.error("unclosed \\p{")
                name, self.i = self.s[self.i + 1:j], j + 1
            else:
                name = self.take_raw() if self.i < len(self.s) else ""
            if name not in POSIX_CLASSES:
                self.error(f"unsupported property \\{c}{{{name}}}")
            if self.ci and name in ("Lower", "Upper"):  # (JDK 8 does not fold these; later JDKs do)
                self.error(f"\\p{{{name}}} under (?i)")
            r = POSIX_CLASSES[name] if c == "p" else cs_neg(POSIX_CLASSES[name])
            return Chars(r) if not in_class else r
        if c == "R" and not in_class:  # Java 8's LineEnding: \r\n taken whole, never given back
            return self._atomic(Alt((Seq((Chars(((13, 13),)), Chars(((10, 10),)))), Chars(VSPACE))))
        if c == "k" and not in_class:  # \k<name>
            j = self.s.find(">", self.i)
            name = self.s[self.i + 1:j] if self.s.startswith("<", self.i) and j > 0 else None
            if name not in self.names:
                self.error("back-reference to an unknown group name")
            self.i = j + 1
            return BackRef(self.names[name])
        if c == "x":
            v = int(self.s[self.i:self.i + 2], 16)
            self.i += 2
        elif c == "u":
            v = int(self.s[self.i:self.i + 4], 16)
            self.i += 4
        elif c == "0":
            # Pattern.o(): one or two octal digits, a third only when the first is 0-3; none is
            # "Illegal octal escape sequence"
            d = self.s[self.i:self.i + 3]
            k = 0
            while k < len(d) and d[k] in "01234567" and (k < 2 or d[0] in "0123"):
                k += 1
            if k == 0:
                self.error("illegal octal escape sequence")
            v = int(d[:k], 8)
            self.i += k
        elif c == "c":
            v = ord(self.take_raw()) ^ 64
        elif c.isdigit() and not in_class:
            return BackRef(int(c))
        elif c in "bB" and not in_class:
            return Anchor("\\b" if c == "b" else "\\B")
        elif c in "AzZ" and not in_class:
            return Anchor({"A": "^", "Z": "$d" if self.unix else "$", "z": "\\z"}[c])
        elif c.isalnum():
            self.error(f"unsupported escape \\{c}")
        else:
            v = ord(c)
        return Chars(self.fold(((v, v),))) if not in_class else ((v, v),)

    def _class_item(self):
        """One plain item of a class (a character, an escape or a range), as code point ranges."""
        c = self.take()
        lo_set = self.escape(in_class=True) if c == "\\" else ((ord(c), ord(c)),)
        if (len(lo_set) == 1 and lo_set[0][0] == lo_set[0][1] and self.peek() == "-"
                and self.i + 1 < len(self.s) and self.s[self.i + 1] not in "[]"):
            self.take()
            d = self.take()
            if d == "\\":
                hi_set = self.escape(in_class=True)
                if len(hi_set) != 1 or hi_set[0][0] != hi_set[0][1]:
                    self.error("class range to a class")
                hi = hi_set[0][0]
            else:
                hi = ord(d)
            if hi < lo_set[0][0]:
                self.error("inverted class range")
            return ((lo_set[0][0], hi),)
        return lo_set

    def char_class(self):
        """A class after its '['.  Nested classes are unions and '&&' intersects what precedes
        with its right operand (one nested class, or plain items up to ']' / '&&'), as Pattern.java
        (JDK 8) parses them; each item is case folded before the sets combine.  A negated class
        holding either is refused: JDK 8 negates only its plain items there (later JDKs the
        whole class), and nothing here pins which one the reference ran."""
        neg = False
        if self.peek() == "^":
            self.take()
            neg = True
        ranges: List[Tuple[int, int]] = []
        acc: Optional[Tuple[Tuple[int, int], ...]] = None  # nested classes / intersections so far
        first = True
        while True:
            c = self.peek()
            if c is None:
                self.error("missing ']'")
            if c == "]" and not first:
                self.take()
                break
            first = False
            if c == "[" or (c == "&" and self.s.startswith("&&", self.i)):
                if neg:
                    self.error("a nested class or && inside a negated class")
                left = cs_norm(list(self.fold(cs_norm(ranges))) + list(acc or ()))
                if c == "[":
                    self.take()
                    acc, ranges = cs_norm(list(left) + list(self.char_class())), []
                    continue
                had_left = bool(ranges) or acc is not None
                self.i += 2
                if self.peek() == "[":
                    self.take()
                    right = self.char_class()
                else:
                    items: List[Tuple[int, int]] = []
                    while self.peek() is not None and self.peek() != "]" and not (
                            self.peek() == "&" and self.s.startswith("&&", self.i)):
                        if self.peek() == "[":
                            self.error("a right operand of && mixing a class and items")
                        items.extend(self._class_item())
                    right = self.fold(cs_norm(items))
                if not (self.peek() == "]" or self.s.startswith("&&", self.i)):
                    self.error("a right operand of && followed by more items")
                acc = cs_and(left, right) if had_left else right
                ranges = []
                continue
            ranges.extend(self._class_item())
        r = self.fold(cs_norm(ranges))  # (case folded before the negation, as Java)
        if acc is not None:
            r = cs_norm(list(r) + list(acc))
        return cs_neg(r) if neg else r


# ------------------------------------------------------------------------------------------------
# AST analysis and rewriting
# ------------------------------------------------------------------------------------------------
def nullable(n) -> bool:
    if isinstance(n, Chars):
        return False
    if isinstance(n, Seq):
        return all(nullable(x) for x in n.items)
    if isinstance(n, Alt):
        return any(nullable(x) for x in n.options)
    if isinstance(n, Repeat):
        return n.lo == 0 or nullable(n.node)
    if isinstance(n, Group):
        return nullable(n.node)
    if isinstance(n, (Look, Anchor, EndText, Behind)):
        return True
    if isinstance(n, BackRef):
        return True  # conservatively (the group may match "")
    raise TypeError(n)


def max_length(n) -> Optional[int]:
    """The most code points a match of `n` spans, or None when unbounded."""
    if isinstance(n, Chars):
        return 1
    if isinstance(n, Seq):
        parts = [max_length(x) for x in n.items]
        return None if any(p is None for p in parts) else sum(parts)
    if isinstance(n, Alt):
        parts = [max_length(x) for x in n.options]
        return None if any(p is None for p in parts) else max(parts, default=0)
    if isinstance(n, Group):
        return max_length(n.node)
    if isinstance(n, Repeat):
        if n.hi == 0:
            return 0
        inner = max_length(n.node)
        return None if n.hi is None or inner is None else n.hi * inner
    if isinstance(n, (Look, Anchor, Behind, EndText)):
        return 0
    return None


def finite_strings(n, limit=64) -> Optional[List[str]]:
    """The finite language of a lookaround-free node, or None (infinite / too many)."""
    if isinstance(n, Chars):
        total = sum(b - a + 1 for a, b in n.ranges)
        if total > limit:
            return None
        return [chr(c) for a, b in n.ranges for c in range(a, b + 1)]
    if isinstance(n, Seq):
        out = [""]
        for x in n.items:
            part = finite_strings(x, limit)
            if part is None:
                return None
            out = [a + b for a in out for b in part]
            if len(out) > limit:
                return None
        return out
    if isinstance(n, Alt):
        out = []
        for x in n.options:
            part = finite_strings(x, limit)
            if part is None:
                return None
            out += part
        return list(dict.fromkeys(out)) if len(out) <= limit else None
    if isinstance(n, Group):
        return finite_strings(n.node, limit)
    if isinstance(n, Repeat):
        if n.hi is None:
            return None
        base = finite_strings(n.node, limit)
        if base is None:
            return None
        out, cur = [], [""]
        for k in range(n.hi + 1):
            if k >= n.lo:
                out += cur
            cur = [a + b for a in cur for b in base]
            if len(out) > limit or len(cur) > limit * limit:
                return None
        return list(dict.fromkeys(out))
    return None


def _literal(s: str):
    return Seq(tuple(Chars(((ord(c), ord(c)),)) for c in s))


def _subst(n, index: int, value: str):
    """Group `index` -> the literal `value`, \\index -> the same literal."""
    if isinstance(n, Group):
        if n.index == index:
            return Group(_literal(value), None)
        return Group(_subst(n.node, index, value), n.index)
    if isinstance(n, BackRef):
        return _literal(value) if n.index == index else n
    if isinstance(n, Seq):
        return Seq(tuple(_subst(x, index, value) for x in n.items))
    if isinstance(n, Alt):
        return Alt(tuple(_subst(x, index, value) for x in n.options))
    if isinstance(n, Repeat):
        return Repeat(_subst(n.node, index, value), n.lo, n.hi)
    if isinstance(n, (Look, Behind)):
        return type(n)(_subst(n.node, index, value), n.negative)
    return n


def _find_group(n, index):
    if isinstance(n, Group):
        if n.index == index:
            return n
        return _find_group(n.node, index)
    for attr in ("items", "options"):
        if hasattr(n, attr):
            for x in getattr(n, attr):
                g = _find_group(x, index)
                if g is not None:
                    return g
    if isinstance(n, (Repeat, Look, Behind)):
        return _find_group(n.node, index)
    return None


def _backrefs(n) -> List[int]:
    if isinstance(n, BackRef):
        return [n.index]
    out = []
    for attr in ("items", "options"):
        if hasattr(n, attr):
            for x in getattr(n, attr):
                out += _backrefs(x)
    if isinstance(n, (Repeat, Look, Group, Behind)):
        out += _backrefs(n.node)
    return out


def expand_backrefs(n):
    """A back-reference to a group with a small finite language (CREDITCARD's separator) becomes a
    union over that language of the pattern with group and reference both set to the value."""
    refs = sorted(set(_backrefs(n)))
    for k in refs:
        g = _find_group(n, k)
        if g is None:
            raise PatternNotSupported(f"back-reference \\{k} to a missing group")
        values = finite_strings(g.node, 16)
        if values is None:
            raise PatternNotSupported(f"back-reference \\{k} to a group with an unbounded language")
        n = Alt(tuple(_subst(n, k, v) for v in values))
    return n


# ------------------------------------------------------------------------------------------------
# Automata over bytes + EOT
# ------------------------------------------------------------------------------------------------
def _utf8_ranges(lo: int, hi: int) -> List[List[Tuple[int, int]]]:
    """Code points [lo, hi] as a union of byte-range sequences (UTF-8, no surrogate check)."""
    out = []
    bounds = [(0, 0x7F, 1), (0x80, 0x7FF, 2), (0x800, 0xFFFF, 3), (0x10000, MAX_CP, 4)]
    for blo, bhi, n in bounds:
        a, b = max(lo, blo), min(hi, bhi)
        if a <= b:
            out += _split(a, b, n)
    return out


def _enc(c: int, n: int) -> List[int]:
    if n == 1:
        return [c]
    if n == 2:
        return [0xC0 | (c >> 6), 0x80 | (c & 0x3F)]
    if n == 3:
        return [0xE0 | (c >> 12), 0x80 | ((c >> 6) & 0x3F), 0x80 | (c & 0x3F)]
    return [0xF0 | (c >> 18), 0x80 | ((c >> 12) & 0x3F), 0x80 | ((c >> 6) & 0x3F), 0x80 | (c & 0x3F)]


def _split(a: int, b: int, n: int) -> List[List[Tuple[int, int]]]:
    if n == 1:
        return [[(a, b)]]
    # split so that all but the first byte span full continuation ranges
    for k in range(1, n):
        m = (1 << (6 * k)) - 1
        if (a & ~m) != (b & ~m):
            if a & m:
                return _split(a, a | m, n) + _split((a | m) + 1, b, n)
            if (b & m) != m:
                return _split(a, (b & ~m) - 1, n) + _split(b & ~m, b, n)
    ea, eb = _enc(a, n), _enc(b, n)
    return [[(x, y) for x, y in zip(ea, eb)]]


class NFA:
    """Thompson-style NFA: trans[s] = list of (symbol bitmask, t); eps[s] = list of t; at0[s] =
    list of t reached without input only at the start of the text (an inner `^`)."""

    def __init__(self):
        self.trans: List[List[Tuple[int, int]]] = []
        self.eps: List[List[int]] = []
        self.at0: List[List[int]] = []
        # (k, t): taken when lookbehind k holds at this position (determinize's `behinds`)
        self.behind: List[List[Tuple[int, int]]] = []
        # (k, t): taken under the obligation that lookahead k holds here (determinize's `aheads`)
        self.ahead: List[List[Tuple[int, int]]] = []

    def new(self) -> int:
        self.trans.append([])
        self.eps.append([])
        self.at0.append([])
        self.behind.append([])
        self.ahead.append([])
        return len(self.trans) - 1


def _mask(lo: int, hi: int) -> int:
    return ((1 << (hi + 1)) - 1) ^ ((1 << lo) - 1)


ALL_BYTES = _mask(0, 255)


class DFA:
    def __init__(self, nxt: List[List[int]], accept: List[bool], start: int):
        self.nxt = nxt        # nxt[state][symbol], symbol in 0..256
        self.accept = accept
        self.start = start

    @property
    def n(self):
        return len(self.nxt)


def determinize(nfa: NFA, start: int, finals: FrozenSet[int], univ: int = -1,
                at_start: bool = True, behinds=(), aheads=()) -> DFA:
    """(behinds: per lookbehind k, (its suffix DFA -- accepting iff the text read so far ends
    with a string of its body -- and whether it is negative); a DFA state is then the NFA subset
    with every suffix DFA's state, and nfa.behind edges are followed where lookbehind k holds.
    aheads: per lookahead k compiled as an obligation (one inside a quantifier), _Ahead.)"""
    if aheads:
        return _determinize_obligations(nfa, start, finals, univ, at_start, behinds, aheads)
    if behinds:
        return _determinize_behind(nfa, start, finals, univ, behinds)
    return _determinize(nfa, start, finals, univ, at_start)


class _Ahead:
    """A lookahead (?=X) / (?!X) as an obligation: the DFA of X Sigma* EOT run from the point it is
    asserted, with the states from which every / no continuation is accepted (it is then decided
    and dropped, or kills its thread)."""

    def __init__(self, d: DFA, negative: bool):
        self.d, self.negative = d, negative
        n = d.n
        good_end = [d.accept[d.nxt[q][EOT]] for q in range(n)]
        rev: List[List[int]] = [[] for _ in range(n)]
        for q in range(n):
            for t in set(d.nxt[q][:256]):
                rev[t].append(q)

        def back(seeds):
            seen, stack = set(seeds), list(seeds)
            while stack:
                for p in rev[stack.pop()]:
                    if p not in seen:
                        seen.add(p)
                        stack.append(p)
            return seen
        may_fail = back([q for q in range(n) if not good_end[q]])
        may_hold = back([q for q in range(n) if good_end[q]])
        self.holds = [q not in may_fail for q in range(n)]  # X has matched: holds for any rest
        self.never = [q not in may_hold for q in range(n)]  # X cannot match any more

    def settle(self, q: int) -> int:
        """0: undecided, 1: the assertion holds, -1: it fails."""
        if self.holds[q]:
            return -1 if self.negative else 1
        if self.never[q]:
            return 1 if self.negative else -1
        return 0


def _determinize_obligations(nfa: NFA, start: int, finals: FrozenSet[int], univ: int,
                             at_start: bool, behinds, aheads) -> DFA:
    """Subset construction over threads (NFA state, obligations): a lookahead edge adds its
    automaton's start state as an obligation of the thread, every symbol advances the thread's
    obligations with it, and a thread dies when one fails (or, at EOT, is not accepted)."""
    def closure(threads, at0, sig):
        stack, seen = list(threads), set(threads)
        while stack:
            s, obl = stack.pop()
            nxt = [(t, obl) for t in nfa.eps[s]]
            if at0:
                nxt += [(t, obl) for t in nfa.at0[s]]
            nxt += [(t, obl) for k, t in nfa.behind[s]
                    if behinds[k][0].accept[sig[k]] != behinds[k][1]]
            for k, t in nfa.ahead[s]:
                a = aheads[k]
                st = a.settle(a.d.start)
                if st >= 0:
                    nxt.append((t, obl if st else obl | {(k, a.d.start)}))
            for x in nxt:
                if x not in seen:
                    seen.add(x)
                    stack.append(x)
        return frozenset(seen)

    def step(threads, sym):
        out = set()
        for s, obl in threads:
            moves = [t for m, t in nfa.trans[s] if (m >> sym) & 1]
            if not moves:
                continue
            kept, ok = [], True
            for k, q in obl:
                a = aheads[k]
                q2 = a.d.nxt[q][sym]
                if sym == EOT:
                    if a.d.accept[q2] == a.negative:
                        ok = False
                        break
                    continue
                st = a.settle(q2)
                if st < 0:
                    ok = False
                    break
                if st == 0:
                    kept.append((k, q2))
            if ok:
                o2 = frozenset(kept)
                out.update((t, o2) for t in moves)
        return out

    sig0 = tuple(d.start for d, _ in behinds)
    none = frozenset()
    u0 = (closure([(univ, none)], False, sig0), ()) if univ >= 0 else None

    def canon(key):
        return u0 if u0 is not None and (univ, none) in key[0] else key

    k0 = canon((closure([(start, none)], at_start, sig0), sig0))
    index = {k0: 0}
    order = [k0]
    nxt, accept = [], []
    i = 0
    while i < len(order):
        cur, sig = order[i]
        i += 1
        accept.append(any(s in finals and not obl for s, obl in cur))
        row = [0] * NSYM
        for sym in range(NSYM):
            sig2 = tuple(d.nxt[q][sym] for (d, _), q in zip(behinds, sig)) if sig else sig
            tgt = step(cur, sym)
            key = canon((closure(tgt, False, sig2), sig2)) if tgt else (frozenset(), ())
            if key not in index:
                if len(order) >= MAX_STATES:
                    raise PatternNotSupported(f"automaton exceeds {MAX_STATES} states")
                index[key] = len(order)
                order.append(key)
            row[sym] = index[key]
        nxt.append(row)
    return DFA(nxt, accept, 0)


def _determinize_behind(nfa: NFA, start: int, finals: FrozenSet[int], univ: int, behinds) -> DFA:
    def closure(states, at_start, sig):
        stack, seen = list(states), set(states)
        while stack:
            s = stack.pop()
            nxt = list(nfa.eps[s]) + (nfa.at0[s] if at_start else [])
            nxt += [t for k, t in nfa.behind[s]
                    if behinds[k][0].accept[sig[k]] != behinds[k][1]]
            for t in nxt:
                if t not in seen:
                    seen.add(t)
                    stack.append(t)
        return frozenset(seen)

    sig0 = tuple(d.start for d, _ in behinds)
    u0 = (closure([univ], False, sig0), ()) if univ >= 0 else None

    def canon(key):
        return u0 if u0 is not None and univ in key[0] else key

    k0 = canon((closure([start], True, sig0), sig0))
    index = {k0: 0}
    order = [k0]
    nxt, accept = [], []
    i = 0
    while i < len(order):
        cur, sig = order[i]
        i += 1
        accept.append(bool(cur & finals))
        edges = [(m, t) for s in cur for m, t in nfa.trans[s]]
        row = [0] * NSYM
        for sym in range(NSYM):
            tgt = frozenset(t for m, t in edges if (m >> sym) & 1)
            sig2 = tuple(d.nxt[q][sym] for (d, _), q in zip(behinds, sig))
            key = canon((closure(tgt, False, sig2), sig2)) if tgt else (frozenset(), ())
            if key not in index:
                if len(order) >= MAX_STATES:
                    raise PatternNotSupported(f"automaton exceeds {MAX_STATES} states")
                index[key] = len(order)
                order.append(key)
            row[sym] = index[key]
        nxt.append(row)
    return DFA(nxt, accept, 0)


def _determinize(nfa: NFA, start: int, finals: FrozenSet[int], univ: int = -1,
                 at_start: bool = True) -> DFA:
    """Subset construction.  `univ` (optional) is a state whose language is everything (Sigma* EOT):
    a subset containing it is that state alone, which keeps the search automaton from tracking
    candidates once one has matched."""
    def closure(states, at_start=False):
        stack, seen = list(states), set(states)
        while stack:
            s = stack.pop()
            for t in nfa.eps[s] + (nfa.at0[s] if at_start else []):
                if t not in seen:
                    seen.add(t)
                    stack.append(t)
        return frozenset(seen)

    u0 = closure([univ]) if univ >= 0 else None

    def canon(t):
        return u0 if u0 is not None and univ in t else t

    s0 = canon(closure([start], at_start=at_start))
    index: Dict[FrozenSet[int], int] = {s0: 0}
    order = [s0]
    nxt: List[List[int]] = []
    accept: List[bool] = []
    i = 0
    while i < len(order):
        cur = order[i]
        i += 1
        accept.append(bool(cur & finals))
        # group the outgoing transitions by symbol
        moves: Dict[int, set] = {}
        edges = [(m, t) for s in cur for m, t in nfa.trans[s]]
        row = [0] * NSYM
        if edges:
            # symbols in play: split by distinct masks
            syms = 0
            for m, _ in edges:
                syms |= m
            for sym in range(NSYM):
                if not (syms >> sym) & 1:
                    continue
                tgt = frozenset(t for m, t in edges if (m >> sym) & 1)
                moves.setdefault(sym, tgt)
        targets: Dict[FrozenSet[int], int] = {}
        for sym in range(NSYM):
            tgt = moves.get(sym)
            if not tgt:
                tset = frozenset()
            else:
                tset = targets.get(tgt)
                if tset is None:
                    tset = canon(closure(tgt))
                    targets[tgt] = tset
            if tset not in index:
                if len(order) >= MAX_STATES:
                    raise PatternNotSupported(f"automaton exceeds {MAX_STATES} states")
                index[tset] = len(order)
                order.append(tset)
            row[sym] = index[tset]
        nxt.append(row)
    return DFA(nxt, accept, 0)


def dfa_to_nfa(d: DFA, nfa: NFA, univ: int) -> Tuple[int, int]:
    """Embeds a DFA (a language of whole remaining texts, EOT included) into an NFA; returns
    (start, final) with eps from accepting states.  States from which every text is accepted
    become the shared universal state `univ`; states from which none is are dropped."""
    n = d.n
    bad = [not d.accept[d.nxt[q][EOT]] for q in range(n)]  # some text (here: the empty one) fails
    live = [d.accept[q] for q in range(n)]
    changed = True
    while changed:
        changed = False
        for q in range(n):
            if not bad[q] and any(bad[d.nxt[q][b]] for b in range(256)):
                bad[q] = changed = True
            if not live[q] and any(live[t] for t in d.nxt[q]):
                live[q] = changed = True
    final = nfa.new()
    base = {}
    for q in range(n):
        if not live[q]:
            continue
        base[q] = univ if not bad[q] else nfa.new()
    for q, node in base.items():
        if node == univ:
            continue
        by_t: Dict[int, int] = {}
        for sym, t in enumerate(d.nxt[q]):
            if t in base:
                by_t[t] = by_t.get(t, 0) | (1 << sym)
        for t, m in by_t.items():
            nfa.trans[node].append((m, base[t]))
        if d.accept[q]:
            nfa.eps[node].append(final)
    if d.start not in base:  # the empty language: a start state with no way out
        return nfa.new(), final
    return base[d.start], final


def product(a: DFA, b: DFA, op) -> DFA:
    index = {(a.start, b.start): 0}
    order = [(a.start, b.start)]
    nxt, acc = [], []
    i = 0
    while i < len(order):
        x, y = order[i]
        i += 1
        acc.append(op(a.accept[x], b.accept[y]))
        row = []
        for sym in range(NSYM):
            p = (a.nxt[x][sym], b.nxt[y][sym])
            if p not in index:
                if len(order) >= MAX_STATES:
                    raise PatternNotSupported(f"automaton exceeds {MAX_STATES} states")
                index[p] = len(order)
                order.append(p)
            row.append(index[p])
        nxt.append(row)
    return DFA(nxt, acc, 0)


def minimize(d: DFA) -> DFA:
    """Moore partition refinement (small automata)."""
    part = [1 if a else 0 for a in d.accept]
    while True:
        sig = {}
        newp = []
        for s in range(d.n):
            key = (part[s], tuple(part[t] for t in d.nxt[s]))
            if key not in sig:
                sig[key] = len(sig)
            newp.append(sig[key])
        if len(sig) == len(set(part)):
            part = newp
            break
        part = newp
    k = max(part) + 1
    nxt = [None] * k
    acc = [False] * k
    for s in range(d.n):
        p = part[s]
        if nxt[p] is None:
            nxt[p] = [part[t] for t in d.nxt[s]]
            acc[p] = d.accept[s]
    return DFA(nxt, acc, part[d.start])


class _Compiler:
    """Thompson construction in continuation-passing style: build(node, s, cont) compiles `node`
    from state s and calls cont(t) exactly once with the state after it (alternatives and
    optional repetitions meet in a join state first), so the rest of the pattern is compiled once.
    A lookahead instead compiles its continuation from a fresh state and records itself; after the
    whole graph exists, lookaheads are resolved right to left: the continuation's DFA (rest of the
    pattern, Sigma*, EOT) combined with X Sigma* EOT (minus for (?! ), intersection for (?= )),
    embedded between s and the final state."""

    def __init__(self):
        self.nfa = NFA()
        self.final = -1
        self._univ = -1
        self.pending: List[Tuple[int, int, object]] = []
        self.behinds: List[Tuple[DFA, bool]] = []  # (suffix DFA, negative) per lookbehind
        self.aheads: List[_Ahead] = []  # lookaheads inside a quantifier, as obligations
        self.loop_depth = 0
        self.all_aheads = False  # every lookahead an obligation (compile_java_regex's retry)

    @property
    def univ(self) -> int:
        """Sigma* EOT -> final (created on first use, after `final`)."""
        if self._univ < 0:
            u = self.nfa.new()
            self.nfa.trans[u].append((ALL_BYTES, u))
            self.nfa.trans[u].append((1 << EOT, self.final))
            self._univ = u
        return self._univ

    def chars(self, ranges, s: int, t: int):
        """s --(one code point in ranges)--> t."""
        for seq in (x for a, b in ranges for x in _utf8_ranges(a, b)):
            cur = s
            for k, (lo, hi) in enumerate(seq):
                nx = t if k == len(seq) - 1 else self.nfa.new()
                self.nfa.trans[cur].append((_mask(lo, hi), nx))
                cur = nx

    def anything(self, s: int) -> int:
        """s --(any bytes)*--> returned state (Sigma* over bytes)."""
        t = self.nfa.new()
        self.nfa.eps[s].append(t)
        self.nfa.trans[t].append((ALL_BYTES, t))
        return t

    def join(self, cont):
        j = self.nfa.new()
        return j, (lambda x: self.nfa.eps[x].append(j))

    def build(self, node, s: int, cont) -> None:
        if isinstance(node, Chars):
            m = self.nfa.new()
            self.chars(node.ranges, s, m)
            cont(m)
        elif isinstance(node, Seq):
            def go(i, st):
                if i == len(node.items):
                    cont(st)
                else:
                    self.build(node.items[i], st, lambda x: go(i + 1, x))
            go(0, s)
        elif isinstance(node, Alt):
            j, to_j = self.join(cont)
            for o in node.options:
                self.build(o, s, to_j)
            cont(j)
        elif isinstance(node, Group):
            self.build(node.node, s, cont)
        elif isinstance(node, Repeat):
            # (a lookbehind or ^ is positional, and a lookahead inside becomes an obligation)
            j, to_j = self.join(cont)
            self.loop_depth += 1

            def rep(k, st):
                if k < node.lo:
                    self.build(node.node, st, lambda x: rep(k + 1, x))
                elif node.hi is None:
                    loop = self.nfa.new()
                    self.nfa.eps[st].append(loop)
                    self.build(node.node, loop, lambda x: self.nfa.eps[x].append(loop))
                    to_j(loop)
                else:
                    to_j(st)
                    if k < node.hi:
                        self.build(node.node, st, lambda x: rep(k + 1, x))
            rep(0, s)
            self.loop_depth -= 1
            cont(j)
        elif isinstance(node, Look) and (self.loop_depth or self.all_aheads):  # an obligation
            if isinstance(node, DollarLook):
                raise PatternNotSupported("$ inside a quantifier")
            x = _Compiler()
            xs = x.nfa.new()
            x.final = x.nfa.new()
            x.build(node.node, xs, lambda st: x.nfa.eps[st].append(x.univ))
            if x.behinds or any(x.nfa.at0):
                raise PatternNotSupported("an anchor or lookbehind inside a lookahead in a quantifier")
            x.resolve_lookaheads()
            d_x = minimize(determinize(x.nfa, xs, frozenset([x.final]), x.univ, aheads=x.aheads))
            t = self.nfa.new()
            self.nfa.ahead[s].append((len(self.aheads), t))
            self.aheads.append(_Ahead(d_x, node.negative))
            cont(t)
        elif isinstance(node, Look):
            mark = self.nfa.new()
            self.pending.append((s, mark, node))  # before cont: lookaheads after it come later
            cont(mark)
        elif isinstance(node, Anchor) and node.kind == "^":  # the start of the text only
            t = self.nfa.new()
            self.nfa.at0[s].append(t)
            cont(t)
        elif isinstance(node, Behind):  # an edge taken where the text so far ends with node
            if _has_look(node.node) or _backrefs(node.node):
                raise PatternNotSupported("a lookaround, anchor or back-reference in a lookbehind")
            if max_length(node.node) is None:  # (Java: "no obvious maximum length")
                raise PatternNotSupported("lookbehind without a bounded length")
            x = _Compiler()
            xs = x.nfa.new()
            x.final = x.nfa.new()
            x.build(node.node, x.anything(xs), lambda st: x.nfa.eps[st].append(x.final))
            d = minimize(determinize(x.nfa, xs, frozenset([x.final])))
            t = self.nfa.new()
            self.nfa.behind[s].append((len(self.behinds), t))
            self.behinds.append((d, node.negative))
            cont(t)
        elif isinstance(node, EndText):  # (in a lookahead: the next symbol ends the text)
            self.nfa.trans[s].append((1 << EOT, self.final))
            cont(self.nfa.new())  # (nothing follows the end)
        elif isinstance(node, Anchor):
            raise PatternNotSupported(f"anchor {node.kind} inside the pattern")
        elif isinstance(node, BackRef):
            raise PatternNotSupported("back-reference")
        else:
            raise TypeError(node)

    def check_inner_anchors(self):
        """Before the lookaheads are resolved: an inner ^ must not follow a lookahead (its
        continuation is compiled as if inside the text), and an inner $ must not follow a byte
        \\r (Java's $ never matches between \\r and \\n; its lookahead would)."""
        nfa = self.nfa
        for s, mark, node in self.pending:
            seen, stack = {mark}, [mark]
            while stack:
                q = stack.pop()
                if nfa.at0[q] or nfa.behind[q]:
                    raise _NeedsObligations("^, \\b or a lookbehind after a lookahead or $ "
                                            "inside the pattern")
                for t in nfa.eps[q] + [t for _, t in nfa.trans[q]] + [t for _, t in nfa.ahead[q]]:
                    if t not in seen:
                        seen.add(t)
                        stack.append(t)
            if isinstance(node, DollarLook):
                pred, stack = {s}, [s]
                while stack:  # states that reach s without input
                    q = stack.pop()
                    for u in range(len(nfa.eps)):
                        if u not in pred and (q in nfa.eps[u] or q in nfa.at0[u] or
                                              any(t == q for _, t in nfa.behind[u])):
                            pred.add(u)
                            stack.append(u)
                for u in range(len(nfa.trans)):
                    if any(t in pred and (m >> 13) & 1 for m, t in nfa.trans[u]):
                        raise _NeedsObligations("$ after a pattern that may end in \\r")

    def resolve_lookaheads(self):
        for s, mark, node in reversed(self.pending):
            # (a continuation starts inside the text: no inner ^ is reachable from it, checked by
            # check_inner_anchors)
            d_cont = minimize(determinize(self.nfa, mark, frozenset([self.final]), self.univ,
                                          at_start=False, aheads=self.aheads))
            x = _Compiler()
            xs = x.nfa.new()
            x.final = x.nfa.new()
            x.build(node.node, xs, lambda st: x.nfa.eps[st].append(x.univ))
            x.resolve_lookaheads()
            d_x = minimize(determinize(x.nfa, xs, frozenset([x.final]), x.univ, aheads=x.aheads))
            op = (lambda p, q: p and not q) if node.negative else (lambda p, q: p and q)
            d = minimize(product(d_cont, d_x, op))
            st, fi = dfa_to_nfa(d, self.nfa, self.univ)
            self.nfa.eps[s].append(st)
            self.nfa.eps[fi].append(self.final)
        self.pending = []


def _has_lookahead(n) -> bool:
    """Whether n holds a lookahead (or an anchor other than ^, which becomes one)."""
    if isinstance(n, Look) or (isinstance(n, Anchor) and n.kind != "^"):
        return True
    if isinstance(n, Behind):
        return False
    for attr in ("items", "options"):
        if hasattr(n, attr) and any(_has_lookahead(x) for x in getattr(n, attr)):
            return True
    if isinstance(n, (Repeat, Group)):
        return _has_lookahead(n.node)
    return False


def _has_look(n) -> bool:
    if isinstance(n, (Look, Anchor, Behind)):
        return True
    for attr in ("items", "options"):
        if hasattr(n, attr):
            if any(_has_look(x) for x in getattr(n, attr)):
                return True
    if isinstance(n, (Repeat, Group)):
        return _has_look(n.node)
    return False


def _may_end_with(node, cp: int) -> bool:
    """Whether some match of `node` can end with code point `cp`."""
    if isinstance(node, Chars):
        return any(a <= cp <= b for a, b in node.ranges)
    if isinstance(node, Seq):
        for x in reversed(node.items):
            if isinstance(x, (Look, Anchor, Behind)):
                continue
            if _may_end_with(x, cp):
                return True
            if not nullable(x):
                return False
        return False
    if isinstance(node, Alt):
        return any(_may_end_with(o, cp) for o in node.options)
    if isinstance(node, Group):
        return _may_end_with(node.node, cp)
    if isinstance(node, Repeat):
        return node.hi != 0 and _may_end_with(node.node, cp)
    return False


def _first_last_word(node, last: bool) -> Optional[bool]:
    """Whether the first (last) code point of every match is a \\b word character (True), never
    one (False), or either (None)."""
    if isinstance(node, Chars):
        word = bound_word_chars()
        inside = all(any(a <= lo and hi <= b for a, b in word) for lo, hi in node.ranges)
        outside = all(all(hi < a or lo > b for a, b in word) for lo, hi in node.ranges)
        return True if inside else (False if outside else None)
    if isinstance(node, Seq):
        items = list(reversed(node.items)) if last else list(node.items)
        for x in items:
            if isinstance(x, (Look, Anchor, Behind)):
                continue
            r = _first_last_word(x, last)
            if nullable(x):
                return None
            return r
        return None
    if isinstance(node, Alt):
        rs = {_first_last_word(o, last) for o in node.options}
        return rs.pop() if len(rs) == 1 else None
    if isinstance(node, (Group,)):
        return _first_last_word(node.node, last)
    if isinstance(node, Repeat):
        return _first_last_word(node.node, last) if node.lo > 0 else None
    return None


@dataclass
class CompiledRegex:
    pattern: str
    n_states: int
    n_classes: int           # byte classes + the EOT class (the last one)
    start: int
    byte_class: bytes        # 256 entries
    accept: bytes            # per state: 0 = undecided, 1 = accepted (sticky), 2 = rejected (dead)
    next: List[int]          # n_states * n_classes, row-major

    def blob(self) -> bytes:
        """Device layout (expr.hip XI_REGEX): int32 n_states, n_classes, start, 0; byte_class[256];
        status[n_states] (padded to 4); uint16 next[n_states * n_classes]."""
        head = struct.pack("<4i", self.n_states, self.n_classes, self.start, 0)
        acc = self.accept + b"\0" * ((-len(self.accept)) % 4)
        nx = struct.pack(f"<{len(self.next)}H", *self.next)
        return head + self.byte_class + acc + nx

    def matches(self, s: str) -> bool:
        """Host run of the same automaton (tests of the compiler itself)."""
        st = self.start
        for b in s.encode("utf-8"):
            if self.accept[st]:
                break
            st = self.next[st * self.n_classes + self.byte_class[b]]
        if not self.accept[st]:
            st = self.next[st * self.n_classes + self.n_classes - 1]
        return self.accept[st] == 1


def compile_java_regex(pattern: str) -> CompiledRegex:
    """Java regex -> DFA over UTF-8 bytes with PatternMatch's find-non-empty semantics."""
    try:
        return _compile_java_regex(pattern, False)
    except _NeedsObligations:
        return _compile_java_regex(pattern, True)


def _compile_java_regex(pattern: str, exact: bool) -> CompiledRegex:
    """exact: every lookahead as an obligation, and $ compiled as Java's Dollar exactly."""
    ast = _Parser(pattern).parse()
    items = list(ast.items) if isinstance(ast, Seq) else [ast]
    start_anchor = end_anchor = None
    # (anchors the edge handling below decides; any other one is an inner anchor)
    if items and isinstance(items[0], Anchor) and items[0].kind in ("^", "\\b"):
        start_anchor = items.pop(0).kind
    if items and isinstance(items[-1], Anchor) and items[-1].kind in (
            ("\\z", "\\b") if exact else ("$", "\\z", "\\b")):
        end_anchor = items.pop().kind
    if nullable(Seq(tuple(items))) and start_anchor in (None, "^") and end_anchor is None:
        # the empty match at offset 0 always succeeds, so find()'s first match starts there:
        # whether it is the non-empty one depends on the match PREFERENCE (greedy / lazy,
        # alternation order), modelled by an ordered-thread automaton
        return compile_nullable(pattern, Seq(tuple(items)))
    body = _rewrite_inner_anchors(expand_backrefs(Seq(tuple(items))), exact=exact)
    if nullable(body):
        raise PatternNotSupported(
            "a pattern that can match the empty string next to an anchor, a lookaround or a "
            "back-reference (the first match need not start at offset 0)")
    c = _Compiler()
    c.all_aheads = exact
    s0 = c.nfa.new()
    c.final = c.nfa.new()
    bound_word = bound_word_chars() if "\\b" in (start_anchor, end_anchor) else WORD
    non_word = cs_neg(bound_word)
    if end_anchor == "$" and _may_end_with(body, 13):
        raise _NeedsObligations("$ after a pattern that may end in \\r")
    # prefix: Sigma*, honouring a leading ^ or \b
    if start_anchor == "^":
        p = s0
    elif start_anchor == "\\b":
        first = _first_last_word(body, last=False)
        if first is None:
            raise PatternNotSupported("\\b before a pattern that may start with either class")
        if first:  # previous code point is a non-word one, or the match starts the row
            p = c.nfa.new()
            c.nfa.eps[s0].append(p)
            any_ = c.anything(s0)
            c.chars(non_word, any_, p)
        else:
            p = c.nfa.new()
            any_ = c.anything(s0)
            c.chars(bound_word, any_, p)
    else:
        p = c.anything(s0)

    def tail(st):
        if end_anchor == "\\z":
            c.nfa.trans[st].append((1 << EOT, c.final))
        elif end_anchor == "$":
            # Java's $ (\Z) also matches before a final line terminator, "\r\n" included
            c.nfa.trans[st].append((1 << EOT, c.final))
            m = c.nfa.new()
            c.chars(LINE_TERMINATORS, st, m)
            c.nfa.trans[m].append((1 << EOT, c.final))
            cr, crlf = c.nfa.new(), c.nfa.new()
            c.chars(((13, 13),), st, cr)
            c.chars(((10, 10),), cr, crlf)
            c.nfa.trans[crlf].append((1 << EOT, c.final))
        elif end_anchor == "\\b":
            last = _first_last_word(body, last=True)
            if last is None:
                raise PatternNotSupported("\\b after a pattern that may end with either class")
            c.nfa.trans[st].append((1 << EOT, c.final) if last else (0, c.final))
            m = c.nfa.new()
            c.chars(non_word if last else bound_word, st, m)
            c.nfa.eps[m].append(c.univ)
        else:
            c.nfa.eps[st].append(c.univ)

    c.build(body, p, tail)
    c.check_inner_anchors()
    c.resolve_lookaheads()
    d = minimize(determinize(c.nfa, s0, frozenset([c.final]), c.univ, behinds=c.behinds,
                             aheads=c.aheads))
    return _finish(pattern, d)


# ------------------------------------------------------------------------------------------------
# Nullable patterns: Java's preferred match at offset 0
#
# A pattern that can match the empty string (and has no anchor but a leading ^, no lookaround, no
# back-reference) always matches at offset 0, so find()'s first match starts there, and the row
# counts iff that match -- the one Java's backtracking prefers -- is non-empty.  Preference is the
# order of Java's backtracking: alternatives left to right, a greedy quantifier's next iteration
# before its exit, a lazy one's exit first, an iteration that consumed nothing not repeated.  A
# leftmost-first Pike program (byte instructions, SPLIT with a preferred branch) simulated with
# threads in priority order finds exactly that match (RE2's leftmost-first semantics, which are
# Perl's and Java's for these constructs); the simulation's states -- the ordered list of live
# threads and whether a match has been recorded at offset 0, later, or not yet -- are finite, and
# become the states of the byte DFA the device runs (the same table format as every pattern).
# ------------------------------------------------------------------------------------------------
_P_BYTE, _P_SPLIT, _P_MATCH, _P_ENTER, _P_BACK = 0, 1, 2, 3, 4


class _Prog:
    """BYTE(mask, next) | SPLIT(preferred, other) | MATCH | ENTER(loop, next) -- an iteration of a
    loop begins | BACK(loop, progressed, empty) -- it ends: continue at `progressed` if it consumed
    input, else at `empty` (Java Pattern.Loop / LazyLoop: an iteration that consumed nothing ends
    the loop, whatever the count)."""

    def __init__(self):
        self.op: List[int] = []
        self.arg: List[list] = []
        self.n_loops = 0

    def emit(self, op, *arg) -> int:
        self.op.append(op)
        self.arg.append(list(arg))
        return len(self.op) - 1

    def choice(self, body: int, exit_: int, greedy: bool) -> int:
        return self.emit(_P_SPLIT, *((body, exit_) if greedy else (exit_, body)))


def _prog_build(prog: _Prog, node, nxt: int) -> int:
    """Compiles `node` to continue at pc `nxt`; returns its entry pc (built back to front, so
    every successor exists when an instruction is emitted)."""
    if isinstance(node, Chars):
        entries = []
        for a, b in node.ranges:
            for seq in _utf8_ranges(a, b):
                pc = nxt
                for lo, hi in reversed(seq):
                    pc = prog.emit(_P_BYTE, _mask(lo, hi), pc)
                entries.append(pc)
        if not entries:  # an empty class matches nothing
            return prog.emit(_P_BYTE, 0, nxt)
        pc = entries[-1]
        for e in reversed(entries[:-1]):  # disjoint byte sequences: the order is immaterial
            pc = prog.emit(_P_SPLIT, e, pc)
        return pc
    if isinstance(node, Seq):
        pc = nxt
        for x in reversed(node.items):
            pc = _prog_build(prog, x, pc)
        return pc
    if isinstance(node, Alt):
        entries = [_prog_build(prog, o, nxt) for o in node.options]
        pc = entries[-1]
        for e in reversed(entries[:-1]):
            pc = prog.emit(_P_SPLIT, e, pc)  # the left alternative first
        return pc
    if isinstance(node, Group):
        return _prog_build(prog, node.node, nxt)
    if isinstance(node, Repeat):
        return _prog_repeat(prog, node, nxt)
    raise PatternNotSupported(f"{type(node).__name__} in a pattern that can match the empty string")


def _prog_repeat(prog: _Prog, node: Repeat, exit_: int) -> int:
    """x{lo,hi} as lo mandatory copies then the optional part (a loop for hi=None, hi-lo nested
    optional copies otherwise).  A body that can match the empty string is bracketed by
    ENTER/BACK so that an empty iteration leaves the repeat (to `exit_`), as in Java."""
    guard = nullable(node.node)
    lid = prog.n_loops
    prog.n_loops += 1

    def copy(progressed: int) -> int:
        if not guard:
            return _prog_build(prog, node.node, progressed)
        back = prog.emit(_P_BACK, lid, progressed, exit_)
        return prog.emit(_P_ENTER, lid, _prog_build(prog, node.node, back))

    if node.hi is None:
        loop = prog.emit(_P_SPLIT, -1, -1)
        body = copy(loop)
        prog.arg[loop] = [body, exit_] if node.greedy else [exit_, body]
        pc = loop
    else:
        pc = exit_
        for _ in range(node.hi - node.lo):
            pc = prog.choice(copy(pc), exit_, node.greedy)
    for _ in range(node.lo):
        pc = copy(pc)
    return pc


def _threads(prog: _Prog, pcs) -> Tuple[int, ...]:
    """The priority-ordered epsilon closure of `pcs` (each started with no loop entered at this
    position): SPLITs take the preferred branch first; a BACK whose loop was ENTERed on the same
    path at this position (the iteration consumed nothing) takes its `empty` exit; BYTE and MATCH
    pcs are kept at their first, highest-priority, occurrence."""
    out: List[int] = []
    kept = set()
    seen = set()
    for start in pcs:
        stack = [(start, frozenset())]
        while stack:
            q, entered = stack.pop()
            op = prog.op[q]
            if op in (_P_BYTE, _P_MATCH):
                if q not in kept:
                    kept.add(q)
                    out.append(q)
                continue
            if (q, entered) in seen:
                continue
            seen.add((q, entered))
            arg = prog.arg[q]
            if op == _P_SPLIT:
                stack.append((arg[1], entered))
                stack.append((arg[0], entered))  # (popped first: the preferred branch)
            elif op == _P_ENTER:
                stack.append((arg[1], entered | {arg[0]}))
            else:  # BACK
                stack.append((arg[2] if arg[0] in entered else arg[1], entered))
    return tuple(out)


def compile_nullable(pattern: str, ast) -> CompiledRegex:
    """The byte DFA of "Java's preferred match at offset 0 is non-empty" (see above)."""
    if _has_look(ast) or _backrefs(ast):
        raise PatternNotSupported("a lookaround or back-reference in a pattern that can match "
                                  "the empty string")
    prog = _Prog()
    match = prog.emit(_P_MATCH)
    start = _prog_build(prog, ast, match)
    # DFA states: (threads, at0, best) -- best: 0 none yet, 1 the empty match, 2 a non-empty one
    ACC, REJ = 0, 1
    states: Dict[Tuple, int] = {}
    table: List[List[int]] = [[ACC] * NSYM, [REJ] * NSYM]
    accept = [True, False]
    work: List[Tuple] = []

    def intern(key) -> int:
        threads, at0, best = key
        if not threads:  # decided
            return ACC if best == 2 else REJ
        if key not in states:
            states[key] = len(table)
            table.append([REJ] * NSYM)
            accept.append(False)
            work.append(key)
            if len(table) > MAX_STATES:
                raise PatternNotSupported(f"automaton exceeds {MAX_STATES} states")
        return states[key]

    def step(threads, at0, best, byte):
        """One position: threads in priority order; a MATCH records the match and cuts every
        lower-priority thread; BYTE threads that take `byte` (None: end of text) advance."""
        nxt = []
        for q in threads:
            if prog.op[q] == _P_MATCH:
                best = 1 if at0 else 2
                break
            if byte is not None and (prog.arg[q][0] >> byte) & 1:
                nxt.append(prog.arg[q][1])
        return _threads(prog, nxt), best

    s0 = intern((_threads(prog, [start]), True, 0))
    while work:
        key = work.pop()
        threads, at0, best = key
        row = table[states[key]]
        for byte in range(256):
            t2, b2 = step(threads, at0, best, byte)
            row[byte] = intern((t2, False, b2))
        _, b_end = step(threads, at0, best, None)
        row[EOT] = ACC if b_end == 2 else REJ
    d = minimize(DFA(table, accept, s0))
    return _finish(pattern, d)


_LINE_END = Alt((Seq((Chars(((13, 13),)), Chars(((10, 10),)))), Chars(LINE_TERMINATORS)))


def _rewrite_inner_anchors(n, in_look: bool = False, consumes_after: bool = False,
                           no_cr_before: bool = False, exact: bool = False):
    """Anchors inside a (non-nullable) pattern: $ and \\Z become the lookahead "at most one
    line terminator, then the end" (DollarLook), \\z the lookahead "the end", ^ and \\A an edge
    taken only at the start of the text (NFA.at0); \\b / \\B the lookbehind-and-lookahead pairs
    of Java's Bound.  exact (every lookahead an obligation): $ and \\Z as Java's Dollar exactly,
    its "never between \\r\\n" a lookbehind."""
    if isinstance(n, Anchor):
        if n.kind == "$":
            if in_look and not no_cr_before:  # (the NFA check below sees only the outer pattern)
                raise PatternNotSupported("$ inside a lookahead, after a possible \\r")
            if exact and not in_look:
                cr, lf = Chars(((13, 13),)), Chars(((10, 10),))
                other = Chars(cs_norm([(13, 13), (0x85, 0x85), (0x2028, 0x2029)]))
                return Alt((Look(EndText(), False),
                            Seq((Behind(cr, True), Look(Seq((lf, EndText())), False))),
                            Look(Seq((other, EndText())), False),
                            Look(Seq((cr, lf, EndText())), False)))
            return DollarLook(Seq((Repeat(_LINE_END, 0, 1), EndText())), False)
        if n.kind == "\\z":
            return Look(EndText(), False)
        if n.kind == "^" and not in_look:
            return n
        # UNIX_LINES / MULTILINE forms (Pattern.java's UnixDollar, Dollar(true), UnixCaret, Caret)
        cr, lf = Chars(((13, 13),)), Chars(((10, 10),))
        if n.kind == "$d":  # the end, or before a final '\n'
            return Look(Seq((Repeat(lf, 0, 1), EndText())), False)
        if n.kind == "$md":  # before any '\n', or at the end
            return Look(Alt((lf, EndText())), False)
        if n.kind == "$m":  # before any line terminator but never between "\r\n", or at the end
            if no_cr_before:  # (the previous character is never '\r': no lookbehind needed)
                return Look(Alt((Chars(LINE_TERMINATORS), EndText())), False)
            if in_look:
                raise PatternNotSupported("$ inside a lookahead, after a possible \\r")
            return Alt((Seq((Behind(cr, True), Look(lf, False))),
                        Look(Chars(cs_norm([(13, 13), (0x85, 0x85), (0x2028, 0x2029)])), False),
                        Look(EndText(), False)))
        if n.kind in ("^m", "^md") and not in_look:
            # the start, or after a line terminator (never between "\r\n"), but not at the end
            if n.kind == "^md":
                after = Behind(lf, False)
            else:
                after = Alt((Behind(Chars(cs_norm([(10, 10), (0x85, 0x85), (0x2028, 0x2029)])), False),
                             Seq((Behind(cr, False), Look(lf, True)))))
            if consumes_after:  # (a character follows in every match: never at the end)
                return Alt((Anchor("^"), after))
            return Seq((Alt((Anchor("^"), after)), Look(Chars(ANY), False)))
        if n.kind in ("\\b", "\\B") and not in_look:  # Java's Bound over \b's word characters
            w = Chars(bound_word_chars())
            b = n.kind == "\\b"  # \b: the two sides differ; \B: they agree
            return Alt((Seq((Behind(w, False), Look(w, b))), Seq((Behind(w, True), Look(w, not b)))))
        raise PatternNotSupported(f"anchor {n.kind} inside the pattern")
    if isinstance(n, Seq):
        def before(k):  # whether the character before item k is never a '\r'
            pre = Seq(n.items[:k])
            return not _may_end_with(pre, 13) and (no_cr_before or not nullable(pre))
        return Seq(tuple(_rewrite_inner_anchors(x, in_look, consumes_after
                                                or not nullable(Seq(n.items[k + 1:])), before(k), exact)
                         for k, x in enumerate(n.items)))
    if isinstance(n, Alt):
        return Alt(tuple(_rewrite_inner_anchors(x, in_look, consumes_after, no_cr_before, exact)
                         for x in n.options))
    if isinstance(n, Group):
        return Group(_rewrite_inner_anchors(n.node, in_look, consumes_after, no_cr_before, exact), n.index)
    if isinstance(n, Repeat):
        return Repeat(_rewrite_inner_anchors(n.node, in_look, exact=exact), n.lo, n.hi, n.greedy)
    if isinstance(n, Behind) and in_look:  # (a lookahead's automaton does not track them)
        raise PatternNotSupported("a lookbehind inside a lookahead")
    if isinstance(n, Look):  # (its body starts where the lookahead stands)
        return Look(_rewrite_inner_anchors(n.node, True, False, no_cr_before, exact), n.negative)
    if isinstance(n, Behind):
        return Behind(_rewrite_inner_anchors(n.node, True, exact=exact), n.negative)
    return n


def _has_anchor(n) -> bool:
    if isinstance(n, Anchor):
        return True
    for attr in ("items", "options"):
        if hasattr(n, attr) and any(_has_anchor(x) for x in getattr(n, attr)):
            return True
    if isinstance(n, (Repeat, Group, Look)):
        return _has_anchor(n.node)
    return False


def _finish(pattern: str, d: DFA) -> CompiledRegex:
    # status: 1 = every continuation accepts (sticky accept), 2 = none does (dead)
    n = d.n
    can_accept = [d.accept[s] for s in range(n)]
    changed = True
    while changed:  # states that reach an accepting state
        changed = False
        for s in range(n):
            if not can_accept[s] and any(can_accept[t] for t in d.nxt[s]):
                can_accept[s] = changed = True
    can_reject = [not d.accept[s] for s in range(n)]
    changed = True
    while changed:
        changed = False
        for s in range(n):
            if not can_reject[s] and any(can_reject[t] for t in d.nxt[s]):
                can_reject[s] = changed = True
    # acceptance happens only on EOT; a state whose EOT successor accepts and from which no input
    # can lead to rejection accepts already
    status = bytearray(n)
    for s in range(n):
        if not can_accept[s]:
            status[s] = 2
        elif not can_reject[s]:
            status[s] = 1
    # byte classes: bytes with identical columns
    cols: Dict[Tuple[int, ...], int] = {}
    byte_class = bytearray(256)
    reps = []
    for b in range(256):
        col = tuple(d.nxt[s][b] for s in range(n))
        if col not in cols:
            cols[col] = len(cols)
            reps.append(b)
        byte_class[b] = cols[col]
    nc = len(cols) + 1
    nxt = []
    for s in range(n):
        nxt += [d.nxt[s][b] for b in reps] + [d.nxt[s][EOT]]
    # EOT always leads to an accepting (status 1 after EOT) or a rejecting state: map the EOT
    # successor's acceptance through its status
    for s in range(n):
        t = d.nxt[s][EOT]
        if d.accept[t]:
            status[t] = 1
    if n > 65535:
        raise PatternNotSupported("automaton too large")
    return CompiledRegex(pattern, n, nc, d.start, bytes(byte_class), bytes(status), nxt)


def nullable_pattern(pattern: str) -> bool:
    ast = _Parser(pattern).parse()
    return nullable(ast)


def accept_all(pattern: str) -> CompiledRegex:
    """Every text matches (RLIKE with a pattern that matches the empty string)."""
    return CompiledRegex(pattern, 1, 2, 0, bytes(256), bytes([1]), [0, 0])


__all__ = ["compile_java_regex", "CompiledRegex", "PatternNotSupported", "nullable_pattern",
           "accept_all"]
