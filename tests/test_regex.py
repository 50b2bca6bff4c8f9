"""The Java-regex -> byte-DFA compiler (deequ_amd/regex.py) against the ORACLE's restatement of
Pattern.find() (oracle/deequ_oracle.py regex_find_nonempty, Python `re`), and the reference's own
PatternMatch known answers (AnalyzerTests.scala:595-688).  Host runs of the compiled automaton
(CompiledRegex.matches, the same table the device walks); no GPU."""
import random
import zlib

import pytest

from deequ_amd.analyzers import Patterns
from deequ_amd.regex import PatternNotSupported, compile_java_regex
from oracle.deequ_oracle import regex_find_nonempty

KNOWN = [  # AnalyzerTests.scala:595-688
    (r"\d", ["1", "a"], 1),
    (Patterns.EMAIL, ["someone@somewhere.org", "someone@else"], 1),
    (Patterns.CREDITCARD, ["378282246310005", "6011111111111117", "6011 1111 1111 1117",
                           "6011-1111-1111-1117", "5555555555554444", "5555 5555 5555 4444",
                           "5555-5555-5555-4444", "4111111111111111", "4111 1111 1111 1111",
                           "4111-1111-1111-1111", "0000111122223333", "000011112222333",
                           "00001111222233"], 10),
    (Patterns.URL, ["http://foo.com/blah_blah", "http://foo.com/blah_blah_(wikipedia)",
                    "http://foo.bar/?q=Test%20URL-encoded%20stuff", "http://\u27a1.ws/\u4a39",
                    "http://\u2318.ws/", "http://\u263a.damowmow.com/", "http://\u4f8b\u5b50.\u6d4b\u8bd5",
                    "https://foo_bar.example.com/", "http://userid@example.com:8080",
                    "http://foo.com/blah_(wikipedia)#cite-1", "http://../", "h://test",
                    "http://.www.foo.bar/"], 10),
    (Patterns.SOCIAL_SECURITY_NUMBER_US, ["111-05-1130", "111051130", "111-05-000", "111-00-000",
                                          "000-05-1130", "666-05-1130", "900-05-1130",
                                          "999-05-1130"], 2),
]


@pytest.mark.parametrize("pattern,rows,expected", KNOWN)
def test_reference_known_answers(pattern, rows, expected):
    c = compile_java_regex(pattern)
    assert sum(c.matches(r) for r in rows) == expected
    assert sum(regex_find_nonempty(r, pattern) for r in rows) == expected  # the oracle too


def _random_strings(rng, alphabet, n, max_len):
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, max_len))) for _ in range(n)]


FUZZ = [
    (Patterns.SOCIAL_SECURITY_NUMBER_US, "0123456789- 9", 14),
    (Patterns.CREDITCARD, "01345679 -x", 22),
    (Patterns.URL, "hftps:/.?#$ a\t\u00e9", 14),
    (Patterns.EMAIL, "ab.@-_[]\"\\1:9", 14),
    (r"a(?!b)c|x{2,3}y?", "abcxy", 8),
    (r"(?:ab|a)(?=c)\w", "abcz_", 7),
    (r"[^\s]+@[\w.]+\.(com|org)$", "a@b.com org\n", 16),
    (r"^\d{2,4}-[A-F]+", "0123-ABFG", 9),
    (r"(x|y)\1z", "xyz", 6),
    (r"\bcat\b", "cat s_", 9),
    (r"caf\u00e9|na.ve|\u4f8b+", "cafe\u00e9nav\u00efi\u4f8b\r", 8),
    # \b next to non-ASCII letters (a word character for Java) and punctuation / currency (not)
    (r"\bab\d\b", "ab1 \u00e9\u20ac\u2014\u00b7\u03b1_x", 8),
    (Patterns.CREDITCARD, "41 -\u00e9\u20ac\u2014\u00d7", 24),
    # Java's $ / \Z before a final "\r\n" or one terminator (never between "\r\n"), \z strict
    (r"a\d$", "a1\r\n\u2028x", 7),
    (r"a\d\Z", "a1\r\n\u0085", 7),
    (r"a\d\z", "a1\r\n", 6),
    # anchors inside the pattern: ^ / \A only at the start of the text, $ / \Z / \z as
    # lookaheads at the end (before one final terminator for $ and \Z)
    (r"(^|,)ab", "ab,x", 7),
    (r"ab($|,)", "ab,\n\r", 7),
    (r"(^|;)[a-c]+($|;)", "abc;d\n", 8),
    (r"x(?:\z|y)", "xy\n", 6),
    (r"(?:\Ab|c)d", "bcd\u2028", 6),
    (r"a(\Z|b)c?", "abc\r\n\u0085", 7),
    (r"(?:q|^)r(?:s|$)", "qrs \n", 6),
    # lookbehind (bounded, as Java requires) and \b / \B inside a pattern: suffix automata run
    # from the text's start beside the subset construction
    (r"(?<=a)b", "abcab ba", 7),
    (r"(?<!a)b", "abcab ba", 7),
    (r"x(?<=ax)y", "axyxyaxy", 8),
    (r"(?<!\d)\d{3}(?!\d)", "1234 567 89x", 10),
    (r"ab\b|cd", "ab cd abx", 8),
    (r"x\By", "xy x y", 6),
    (r"\b\d+\b ", "12 3a 45 ", 9),
    # embedded flags: DOTALL, UNIX_LINES, MULTILINE (Pattern.java's Caret / Dollar(true) and their
    # UNIX_LINES forms, never between "\r\n"), COMMENTS (white space and #-comments ignored,
    # inside classes too), each scoped to its group as (?i) is
    (r"(?s)a.b", "ab\r\n\x85\u2028x", 6),
    (r"(?d)a.b", "ab\r\n\x85x", 6),
    (r"a(?s:.)b|c.d", "abcd\n\r", 6),
    (r"(?m)^ab", "ab\r\nx\x85\u2028", 8),
    (r"(?m)ab$", "ab\r\nx\x85\u2029", 8),
    (r"(?m)^a+$", "ab\r\n\x85", 8),
    (r"(?m)x\r$", "x\r\n", 6),
    (r"(?m)(?:^|,)a(?:,|$)", "a,\n\rb", 8),
    (r"(?md)^ab$", "ab\r\nx", 8),
    (r"(?d)ab$|c\Z", "abc\r\nx", 6),
    (r"(?x) a b # c", "ab #c", 6),
    (r"(?x)[a b]c", "abc ", 6),
    (r"(?x)a\ b|(?-x: c)", "abc ", 6),
    (r"(?is)A.B|(?-i)c", "aAbBcC\n", 6),
    (r"((?m)^a|b)$", "ab\n", 6),
    (r"(?m)^\s*#", " #\n\r\x85a", 8),
    # the US-ASCII POSIX classes \p{...} / \P{...}, \h \v, \Q...\E (Pattern.java's
    # RemoveQEQuoting: a quantifier binds to the last quoted character), named groups
    (r"\p{Alpha}+\d", "aZ1 _\u00e9", 6),
    (r"[\p{Punct}\h]x", "!x ~ \t_\u3000", 5),
    (r"\P{Digit}a|\p{XDigit}{2}\p{Space}", "1a 0F\n", 6),
    (r"\QA.b\E+|x\Q(*)\E", "A.bxB(*)", 6),
    (r"(?<sep>[-/])\d\k<sep>\d", "-/1", 6),
    (r"\va\V", "a\n\r\x85 x", 5),
    (r"(?x)\p{Upper} \Q a b\E", "A ab", 7),
    # lookaheads inside a quantifier (obligations carried by each thread of the subset
    # construction), lookbehinds and ^ inside one (positional)
    (r"a(?:(?!b).)*c", "abcx", 8),
    (r"a(?:(?!bc).)+d", "abcdx", 9),
    (r"<(?:(?!<).)*>", "<a>b<", 8),
    (r"(?:\w(?=\d))+\d", "a1b2_", 8),
    (r"(?:a\b)+", "a b", 6),
    (r"q(?:(?!x|yz)[xyz])*q", "qxyz", 8),
    (r"(?:a(?=b|$))+", "ab\n\r", 6),
    (r"(?=a)(?:a(?!a))+b", "ab", 6),
    (r"(?:(?<=a)b)+c", "abc", 7),
    (r"(?m)(?:^a)+|x(?:(?<![0-9])[a-c])*y", "a\nbxy1c", 8),
    # what the lookahead product refuses, compiled again with every lookahead an obligation and $
    # as Java's Dollar exactly (never between "\r\n"): $ after a possible \r, ^ / lookbehind /
    # \b after a lookahead
    (r"a\s$", "a \r\n", 6),
    (r"(?:a|\r)$x?", "a\r\nx", 6),
    (r"(?:a(?!b)|\r)+$", "ab\r\n", 6),
    (r"(?sm)^.+$", "ab\r\n", 6),
    (r"[^x]+$", "ax\r\n\x85", 6),
    (r"(?=a)(^|b)a", "ab", 5),
    (r"(?=a)a(?<=a)b|(?=a)a\bb", "ab ", 5),
    (r"(?=.*\d)\w+\r$", "a1\r\n", 6),
    # class set operations (JDK 8 Pattern.clazz): nested classes are unions, && intersects
    (r"[a-z&&[^aeiou]]{2}", "abeiz1", 6),
    (r"x[a-d[m-p]]y", "xaymyzy", 6),
    (r"[\w&&[^\d_]]+\d", "a1_Z9 ", 6),
    (r"[a-z&&def]!|[abc&&b-d&&[^c]]", "abcdf!", 5),
    (r"(?i)[a-c&&[B-Z]]x", "aAbBcCx", 5),
    (r"[[a-c][x-z]&&[^by]]q|[\p{Alpha}&&[^a-f]][a[b]c]", "abcxyzqfg", 5),
    # possessive quantifiers over one character class: C{lo,}(?!C), C{hi} | C{lo,hi-1}(?!C)
    (r"a*+a|[a-z]++\d", "ab1 ", 6),
    (r'"[^"]*+"', 'a""b', 6),
    (r"\d{2,4}+5", "1235x", 7),
    (r"b(?:a++|c)+d|x?+x", "abcdxy", 7),
    (r"(?i)A++b|[ab]{1,3}+b", "aAbB", 6),
    # atomic groups: one class repeated (the possessive form), or a finite language as "s_k where
    # no earlier s_j (backtracking order) starts here"
    (r"(?>ab|a)b|(?>a|ab)c", "abc", 6),
    (r"x(?>a*)a|x(?>a+?)a", "xa", 6),
    (r"(?>(?:a|ab){0,2})c", "abc", 7),
    (r"(?>[0-9]{1,3})5|(?i)(?>A|B)c", "0159aAbBcC", 6),
    (r"(?>a?b?)c|q|(?>x(?:y|yz))z", "abcqxyz", 6),
    (r"(?>ab|a){2}b", "ab", 7),
    # \R: JDK 8's LineEnding, "\r\n" taken whole and never given back
    (r"a\R\n|a\Rb", "ab\r\n\x0b\x85", 6),
    (r"\R{2}x", "\r\nx\u2028", 6),
]


@pytest.mark.parametrize("pattern,alphabet,max_len", FUZZ)
def test_automaton_matches_java_find_semantics(pattern, alphabet, max_len):
    rng = random.Random(zlib.crc32(pattern.encode()))
    c = compile_java_regex(pattern)
    for s in _random_strings(rng, alphabet, 3000, max_len):
        assert c.matches(s) == regex_find_nonempty(s, pattern), (pattern, s)


# Patterns that can match the empty string: the row counts iff Java's PREFERRED match at offset 0
# is non-empty (greedy / lazy, alternation order, an empty iteration ending its loop), and the case
# flag (?i) scoped to its group
NULLABLE = [
    (r"\d*", "12a 3", 7),
    (r"\d*?", "12a", 5),
    (r"(?i)http", "hHtTpPs:", 7),
    (r"(?i)ab*|c", "aAbBcC", 6),
    (r"a(?i)b|c", "aAbBcC", 6),
    (r"x(?i:y)z", "xXyYzZ", 6),
    (r"(?i)[^a-c]x", "aAbBxXdD", 6),
    (r"[0-9]*(\.[0-9]+)?", "12.3.a", 8),
    (r"(a|ab)*c?", "abc", 8),
    (r"(ab|a)*?b?", "abc", 8),
    (r"(?:a??)+b?", "abx", 6),
    (r"(a?){2,}b?", "abx", 6),
    (r"(a?){1,3}?b", "abx", 6),
    (r"(|a)b?", "abx", 5),
    (r"^\s*\w*", " \tab_1-", 8),
    (r"(?:x|\u00e9)*y?", "x\u00e9y\u00c9", 6),
]


@pytest.mark.parametrize("pattern,alphabet,max_len", NULLABLE)
def test_nullable_patterns_match_javas_preferred_match(pattern, alphabet, max_len):
    rng = random.Random(zlib.crc32(pattern.encode()))
    c = compile_java_regex(pattern)
    for s in [""] + _random_strings(rng, alphabet, 3000, max_len):
        assert c.matches(s) == regex_find_nonempty(s, pattern), (pattern, s)


def test_nullable_known_answers():
    # Java: "12ab".find(\d*) -> "12"; "ab12" -> "" at 0; lazy \d*? -> "" always
    assert [compile_java_regex(r"\d*").matches(s) for s in ["12ab", "ab12", ""]] == [True, False, False]
    assert not compile_java_regex(r"\d*?").matches("123")
    assert [compile_java_regex(r"(?i)http").matches(s) for s in ["HTTP", "xHtTp", "htp"]] == [True, True, False]
    # an empty first iteration ends Java's loop: (?:a??)+ prefers "" and never iterates again
    assert not compile_java_regex(r"(?:a??)+b?").matches("ab")


@pytest.mark.parametrize("pattern", [r"(?:ab)++", r"(?>a+b)", r"a*$", r"(?=x)a*", r"(a?)\1",
                                     # Unicode case folding / character classes
                                     r"(?iu)a", r"(?U)\w", r"(?m)^$",
                                     # Unicode properties, \p{Lower} / \p{Upper} under (?i)
                                     r"\pL", r"\p{IsDigit}", r"(?i)\p{Lower}",
                                     # $ in a lookahead after a possible \r, a lookbehind in one
                                     r"\r(?=$)", r"a(?=\r$)", r"(?=(?<=a)b)b",
                                     # lookbehinds: unbounded (Java refuses it too), holding a
                                     # lookaround
                                     r"(?<=a+)b", r"(?<=(?=a)a)b",
                                     # set operations in a negated class (JDK 8 negates only
                                     # its plain items), a mixed right operand of &&
                                     r"[^a[b]]", r"[^a&&b]", r"[a&&[b]c]"])
def test_unsupported_patterns_are_refused(pattern):
    with pytest.raises(PatternNotSupported):
        compile_java_regex(pattern)


def test_octal_escapes_and_quoted_digits_as_jdk8():
    # Pattern.o(): a third octal digit only after a first digit 0-3; \0 with none is illegal
    assert compile_java_regex(r"\0101").matches("xA")            # 0101 = 'A'
    c = compile_java_regex(r"\0477")                              # 047 = "'", then a literal 7
    assert c.matches("'7") and not c.matches("\u0137")
    # RemoveQEQuoting writes a digit first in a \Q section as \x3N: no escape absorbs it
    c = compile_java_regex(r"(a)\Q1\E")                           # not the back-reference \11
    assert c.matches("a1") and not c.matches("aa")
    assert compile_java_regex(r"\Q12\E").matches("x12")
    for bad in [r"\0", r"\0x", r"\08", r"\0\Q1\E"]:                      # Java: Illegal octal escape
        with pytest.raises(PatternNotSupported):
            compile_java_regex(bad)


def test_blob_layout():
    c = compile_java_regex(r"\d")
    b = c.blob()
    import struct
    ns, nc, start, zero = struct.unpack_from("<4i", b)
    assert (ns, nc, start, zero) == (c.n_states, c.n_classes, c.start, 0)
    assert len(b) == 16 + 256 + ((ns + 3) & ~3) + 2 * ns * nc
