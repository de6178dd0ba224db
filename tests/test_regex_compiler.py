"""Chain-build-time regex -> byte-DFA compiler (host code of libfsg.so),
checked against the oracle's independent Pike-VM engine and Python `re`."""
import ctypes
import random

import pytest

from fluvio_amd import _ffi
from oracle import oracle as O


def dfa_match(pattern, text):
    m, ml, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = _ffi.debug_lib().fsg_debug_regex_match(pattern.encode(), text, len(text), ctypes.byref(m),
                                          ctypes.byref(ml), ctypes.byref(ns))
    if rc:
        raise ValueError(rc)
    return bool(m.value), ml.value, ns.value


PATTERNS = [r"\d{3}-\d{2}-\d{4}", r"[A-Z]", r"^ab|cd$", r"a(b|c)*d", r"colou?r\s+x", r"[^a-c]x", r"a.c",
            r"x{2,3}y", r"", r"^$", r"^a", r"b$", r"timeout", r"(?:ab)+c", r"[0-9a-f]{4}", r"\s\S\d\D",
            r"é+", r"[α-ω]{2}", r".{3}$", r"(a|ab)(c|bcd)(d*)", r"a?a?a?aaa", r"\x41\x{263A}", r"[\-\]a]",
            r"\bab", r"cd\b", r"\b\d+\b", r"\Ba\B", r"x\b|\by", r"\b", r"(?i)abcd", r"(?i)[a-c]x|D$",
            r"(?i:ab)c", r"(?i)[^a]", r"(?s)a.c", r"\Aab", r"cd\z", r"[[:alpha:]]{3}", r"[[:^digit:][:space:]]x",
            r"(?i)[[:lower:]]{2}\b", r"\w+é", r"^\w+$", r"\W\w", r"[\w-]{3}", r"\p{Lu}", r"\P{L}\pN",
            r"\p{gc=Nd}", r"[\p{Sc}\d]", r"\p{^Ll}", r"(?m)^b$", r"(?m)a$|^c", r"(?m:^)x|y(?-m)$",
            r"(?x) a b # comment", r"(?x)[ a ] c", r"(?x: \d \  \d )", r"(?-u)\w\d\s", r"(?u)\w(?-u:[a-z])",
            # nested classes, class set operations, \u / \U escapes
            r"[a-z&&[^aeiou]]{2}", r"[\w--\d]+x", r"[a-g~~c-j]", r"[0-9--4]", r"[[a-c][x-z]]", r"[^[a-c]d]",
            r"[a-z&&b-y&&[^m]]", r"[\pL&&\p{Ll}]é", r"[\p{L}--[a-zé]]", r"[a-c~~b-d~~c-e]", r"[--a]", r"[]a]",
            r"[a-c--b]d", r"\u0041\U0001F600?\u{263a}", r"[\u00e9-\u00ea\U000003b1]", r"(?i)[a-z--k]",
            r"(?-u)[[^a]&&[b-c]]", r"(?x)[ a-z && [^ x ] ]",
            # binary properties, scripts, Script_Extensions; (?i) on Unicode literals and classes
            r"\p{Greek}+", r"\p{sc=Cyrillic}\w", r"\p{scx=Grek}", r"\p{Alphabetic}{2}", r"\p{Emoji}",
            r"\P{Greek}$", r"[\p{Greek}&&\p{Ll}]", r"\p{Script_Extensions=Arabic}", r"\p{Upper}\p{Lower}",
            r"\p{White_Space}", r"(?i)\p{Lu}", r"(?i)é", r"(?i)Σ", r"(?i)[α-γ]x?", r"(?i)ǆ", r"(?i)\P{Ll}",
            r"(?i)[^σ]", r"(?i)ж+", r"(?i)[\p{Greek}--α]",
            # Unicode word boundaries on non-ASCII text (the marked full DFA)
            r"\bαβ", r"ω\b", r"\b\w+\b", r"é\B", r"\B☺", r"(?m)^\bЖ|ж\b$", r"(?i)\bσ\b", r"\b[α-ω]{2}\b"]
WORD = ("\\b", "\\B")


def texts(rng):
    alpha = "abcdxyzABCD0123456789- \t\n.é☺αβωÉ٣€_#ΣσςЖжǄǅǆΑΓ"
    out = ["", "a", "abc", "ac", "xxy", "123-45-6789", "my ssn 987-65-4321!", "colour  x", "☺A", "aé",
           "abcd", "cd", "ab", "timeouts", "αβγ", "aaa", "abcbcd", "a\nb\nc", "x\nb", "naïve", "9 ٣", "c\na"]
    for _ in range(60):
        out.append("".join(rng.choice(alpha) for _ in range(rng.randint(0, 24))))
    return out


@pytest.mark.parametrize("pattern", PATTERNS)
def test_dfa_matches_oracle(pattern):
    rng = random.Random(hash(pattern) & 0xFFFF)
    word = any(w in pattern for w in WORD)
    for t in texts(rng):
        b = t.encode()
        if word and not b.isascii() and "(?-u" in pattern:  # a (?-u) \b: UNSUPPORTED on non-ASCII values
            with pytest.raises(ValueError):
                dfa_match(pattern, b)
            continue
        assert dfa_match(pattern, b)[0] == O.regex_is_match(pattern, b), (pattern, t)


def test_max_len():
    assert dfa_match(r"\d{3}-\d{2}-\d{4}", b"")[1] == 11
    assert dfa_match(r"a+", b"")[1] == -1
    assert dfa_match(r"é", b"")[1] == 0  # ASCII DFA: the class is empty on ASCII values


@pytest.mark.parametrize("bad,code", [("a(", _ffi.FSG_E_INIT), ("*a", _ffi.FSG_E_INIT), ("[z-a]", _ffi.FSG_E_INIT),
                                      ("(?)a", _ffi.FSG_E_INIT), ("(?z)a", _ffi.FSG_E_INIT), ("[\\b]", _ffi.FSG_E_INIT),
                                      ("(?-u:.)", _ffi.FSG_E_INIT), ("(?-u)[^a]", _ffi.FSG_E_INIT),
                                      (r"(?-u)\W", _ffi.FSG_E_INIT), (r"(?-u)\pL", _ffi.FSG_E_INIT),
                                      (r"\p{", _ffi.FSG_E_INIT), (r"\p{Nope}", _ffi.FSG_E_INIT),
                                      (r"\p{Age=3.0}", _ffi.FSG_E_UNSUPPORTED), ("(?R)a", _ffi.FSG_E_UNSUPPORTED),
                                      (r"\p{CWKCF}", _ffi.FSG_E_UNSUPPORTED), (r"\p{Garay}", _ffi.FSG_E_INIT),
                                      ("[a-c", _ffi.FSG_E_INIT), ("[a[b]", _ffi.FSG_E_INIT), (r"\u12", _ffi.FSG_E_INIT),
                                      (r"\u{110000}", _ffi.FSG_E_INIT), (r"\ud800", _ffi.FSG_E_INIT),
                                      (r"(?-u)[[^a]--b]", _ffi.FSG_E_INIT)])
def test_errors_agree_with_oracle(bad, code):
    with pytest.raises(ValueError) as e:
        dfa_match(bad, b"x")
    assert e.value.args[0] == code
    with pytest.raises(ValueError):
        O.regex_is_match(bad, b"x")


def _random_pattern(rng, depth=0):
    atoms = ["a", "b", "é", "α", ".", r"\d", r"\w", r"\W", r"\s", r"\pL", r"\p{Lu}", r"\P{N}", "[a-cé]", "[^b]",
             r"[\w-]", r"[α-ω\d]", "^", "$", r"\x{263A}", "(?m:^)", "(?m:$)", "(?i:ab)", "(?s:.)",
             r"[\w&&[^a\d]]", r"[[a-c]--b]", r"[é~~\pL]", r"[^[α-ω]&&\pL]", r"\u00e9"]
    if depth > 2 or rng.random() < 0.4:
        a = rng.choice(atoms)
    elif rng.random() < 0.5:
        a = "(?:" + "|".join(_random_pattern(rng, depth + 1) for _ in range(rng.randint(1, 3))) + ")"
    else:
        a = "(?:" + "".join(_random_pattern(rng, depth + 1) for _ in range(rng.randint(1, 3))) + ")"
    if a not in ("^", "$", "(?m:^)", "(?m:$)"):
        a += rng.choice(["", "", "*", "+", "?", "{2}", "{1,3}", "*?"])
    return a


def test_random_patterns_match_oracle():
    """Random patterns over Unicode classes, properties, multi-line anchors and
    repeats: the minimized byte DFA decides exactly what the Pike VM decides.
    A pattern whose DFA exceeds the chain-build budget is FSG_E_UNSUPPORTED
    (loud, never a wrong answer); those must stay the exception."""
    rng = random.Random(7)
    alpha = "abéαβA1 \n-☺_٣É"
    n = too_large = 0
    for _ in range(150):
        pat = "".join(_random_pattern(rng) for _ in range(rng.randint(1, 3)))
        tx = ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 10))).encode() for _ in range(12)]
        try:
            dfa_match(pat, b"")
        except ValueError as e:
            assert e.args[0] == _ffi.FSG_E_UNSUPPORTED, pat
            too_large += 1
            continue
        for t in tx:
            assert dfa_match(pat, t)[0] == O.regex_is_match(pat, t), (pat, t)
            n += 1
    assert n > 1000 and too_large < 20, (n, too_large)


@pytest.mark.parametrize("pattern,text,expect", [
    # (?i) folds KELVIN SIGN / LONG S to k / s only in Unicode mode; (?-u) folds ASCII bytes
    (r"(?i)k", "K", True), (r"(?i-u)k", "K", False), (r"(?i)s", "ſ", True),
    (r"(?i-u)s", "ſ", False), (r"(?i-u)[[:alpha:]]", "K", False), (r"(?i-u)K", "k", True),
    (r"(?i)[[:alpha:]]", "K", True),
    # simple case folding (CaseFolding C + S): orbits, no full folding, no Turkic entries
    (r"(?i)σ", "ς", True), (r"(?i)Σ", "σ", True), (r"(?i)ß", "ẞ", True), (r"(?i)^ß$", "ss", False),
    (r"(?i)i", "ı", False), (r"(?i)i", "İ", False), (r"(?i)I", "i", True), (r"(?i)ǆ", "ǅ", True),
    (r"(?i)ǆ", "Ǆ", True), (r"(?i)θ", "ϑ", True), (r"(?i)\p{Lu}", "a", True), (r"\p{Lu}", "a", False),
    (r"(?i)[^a]", "A", False), (r"(?i)\P{Lu}", "A", False), (r"(?i)\P{Lu}", "a", False), (r"(?i)\P{Lu}", "1", True), (r"(?i)ω", "Ω", True), (r"(?i)µ", "Μ", True),
    (r"\p{Greek}", "ω", True), (r"\p{Greek}", "w", False), (r"\p{sc=Latin}", "é", True),
    (r"\p{isGreek}", "ω", True),
    # (?x): whitespace around a class range's '-' is skipped (parse_set_class_range's bump_space)
    (r"(?x)[a - z]", "m", True), (r"(?x)[a - z]", "-", False), (r"(?x)[a - ]", "-", True),
    (r"(?x)[ a -z ]x", "qx", True), (r"[a - z]", "-", False), (r"[a - z]", " ", True), (r"[a - z]", "m", False),
    # the "is" prefix is dropped from the raw part only ("I_s" is not a prefix; "isc" = ISO_Comment, not "c")
    (r"\p{IsLu}", "A", True), (r"\p{IsLu}", "a", False), (r"\p{sc=IsArabic}", "\u0628", True),
    (r"\p{sc=IsArabic}", "b", False), (r"\p{IsScript:Greek}", "\u03c9", True), (r"\p{I_sGreek}", "x", None), (r"\p{Isc}", "x", None),
])
def test_fold_and_x_ranges(pattern, text, expect):
    b = text.encode()
    if expect is None:  # a name regex-syntax does not resolve: Regex::new fails (an init error) on both sides
        with pytest.raises(ValueError):
            O.regex_is_match(pattern, b)
        with pytest.raises(ValueError) as e:
            dfa_match(pattern, b)
        assert e.value.args[0] == _ffi.FSG_E_INIT
        return
    assert O.regex_is_match(pattern, b) == expect
    assert dfa_match(pattern, b)[0] == expect


@pytest.mark.parametrize("pattern", [r"\p{Greek}", r"\p{Cyrillic}+", r"\p{scx=Arabic}", r"\p{Emoji}", r"\p{Alphabetic}",
                                     r"\p{Uppercase}", r"\p{Dash}", r"\p{Han}", r"\P{Latin}", r"[\p{Greek}\p{Cyrillic}]{2}",
                                     r"\p{Extended_Pictographic}", r"\p{Math}",
                                     # symbolic_name_normalize's "is" prefix, per part of name=value
                                     r"\p{IsGreek}", r"\p{Is_Cyrillic}", r"\p{IsAlphabetic}",
                                     r"\p{IsHan}+",
                                     # Grapheme_Cluster_Break / Word_Break / Sentence_Break values
                                     r"\p{GCB=Extend}", r"\p{Grapheme_Cluster_Break=Other}{2}", r"\p{WB=ALetter}+",
                                     r"\p{Word_Break=Numeric}", r"\p{SB=Upper}", r"\P{Sentence_Break=Lower}",
                                     r"\p{gcb=EB}", r"[\p{WB=MidLetter}\p{WB=Katakana}]"])
def test_properties_against_python_regex(pattern):
    """Binary properties, scripts and Script_Extensions over random text of
    Greek, Cyrillic, Latin, Arabic, CJK and symbols, against Python's `regex`
    module (the tables' source: the same UCD values)."""
    regex = pytest.importorskip("regex")
    rng = random.Random(hash(pattern) & 0xFFFF)
    alpha = "aZé-ωΣж٣ب漢☺€+𝟘😀́ 1_"
    for _ in range(200):
        t = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 6)))
        want = regex.search(pattern, t) is not None
        assert dfa_match(pattern, t.encode())[0] == want, (pattern, t)
        assert O.regex_is_match(pattern, t.encode()) == want, (pattern, t)


@pytest.mark.parametrize("bad", [r"(?-u)[é]", r"(?-u)[a-é]", r"(?-u)[é]"])
def test_non_ascii_class_literal_without_unicode(bad):
    """class_literal_byte: a literal outside ASCII in a (?-u) class is
    UnicodeNotAllowed (an init error); outside a class it stays a literal."""
    with pytest.raises(ValueError) as e:
        dfa_match(bad, b"x")
    assert e.value.args[0] == _ffi.FSG_E_INIT
    with pytest.raises(ValueError):
        O.regex_is_match(bad, b"x")
    assert dfa_match(r"(?-u)é", "é".encode())[0] and O.regex_is_match(r"(?-u)é", "é".encode())


@pytest.mark.parametrize("pattern", [r"[a-z&&[^aeiou]]", r"[a-y&&xyz]", r"[0-9--4]", r"[a-g~~b-h]", r"[\w--\d]",
                                     r"[[a-c][x-z]]x", r"[^[a-c]d]", r"[a-z--[b-y]&&[^z]]", r"[a-c~~b-d~~c-e]",
                                     r"[0-9&&[^4]]{2}", r"\u0041b", r"[\u0061-\u0063]z"])
def test_set_operations_against_python_regex(pattern):
    """regex-syntax's class set operations / nested classes / \\u escapes on ASCII
    text, against Python's `regex` module (V1 set syntax, the same grammar on
    these patterns): the DFA and the oracle agree with it."""
    regex = pytest.importorskip("regex")
    rng = random.Random(hash(pattern) & 0xFFFF)
    for _ in range(200):
        t = "".join(rng.choice("abcdefghmxyz0459AZ_-") for _ in range(rng.randint(0, 6)))
        want = regex.search("(?V1)" + pattern, t) is not None
        assert dfa_match(pattern, t.encode())[0] == want, (pattern, t)
        assert O.regex_is_match(pattern, t.encode()) == want, (pattern, t)


@pytest.mark.parametrize("pattern", [r"\bαβ", r"ω\b", r"\b\w+\b", r"é\B", r"\B☺", r"\b[α-ω]{2}\b", r"\bx", r"x\b",
                                     r"\b٣", r"\B\d"])
def test_unicode_word_boundaries_against_python_regex(pattern):
    """\\b / \\B between code points by Unicode \\w (the marked DFA, and the
    oracle's Pike VM over code points), against Python's `regex` module."""
    regex = pytest.importorskip("regex")
    rng = random.Random(hash(pattern) & 0xFFFF)
    alpha = "xaé ωαβ☺٣-_ж́.1"
    for _ in range(300):
        t = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 7)))
        want = regex.search(pattern, t) is not None
        assert dfa_match(pattern, t.encode())[0] == want, (pattern, t)
        assert O.regex_is_match(pattern, t.encode()) == want, (pattern, t)


def regex_error(pattern):
    buf = ctypes.create_string_buffer(8192)
    rc = _ffi.debug_lib().fsg_debug_regex_error(pattern.encode(), buf, len(buf))
    return rc, buf.value.decode()


TILDES = "~" * 79


@pytest.mark.parametrize("pattern,text", [
    # regex-syntax's Formatter (error.rs, the same in 0.6.27 and 0.7.1): the
    # span of a \p class under the one-line pattern, "error: <ErrorKind Display>"
    (r"\p{Garay}", "regex parse error:\n    \\p{Garay}\n    ^^^^^^^^^\nerror: Unicode property not found"),
    (r"a\p{sc=Garay}b",
     "regex parse error:\n    a\\p{sc=Garay}b\n     ^^^^^^^^^^^^\nerror: Unicode property value not found"),
    (r"é[\w\p{bc=L}]", "regex parse error:\n    é[\\w\\p{bc=L}]\n        ^^^^^^^^\nerror: Unicode property not found"),
    (r"\pQ", "regex parse error:\n    \\pQ\n    ^^^\nerror: Unicode property not found"),
    (r"\p{gc=Nope}|\p{Nope}",
     "regex parse error:\n    \\p{gc=Nope}|\\p{Nope}\n    ^^^^^^^^^^^\nerror: Unicode property value not found"),
    # a pattern with a newline: numbered lines between two rules of 79 '~'
    ("x\n\\p{Nope}+\ny",
     "regex parse error:\n" + TILDES + "\n1: x\n2: \\p{Nope}+\n   ^^^^^^^^\n3: y\n" + TILDES +
     "\nerror: Unicode property not found"),
])
def test_property_init_error_text(pattern, text):
    """Where regex-syntax rejects a \\p name at Regex::new (an unknown property
    or value, a script of Unicode 16+), the library's init error carries the
    regex crate's Display of that error, and the oracle's is the same text;
    the expected strings are written from regex-syntax's formatter (parity
    unpinned: no reference fixture holds such an error)."""
    rc, msg = regex_error(pattern)
    assert rc == _ffi.FSG_E_INIT
    assert msg == text
    with pytest.raises(O.OracleError) as e:
        O.OracleChain([("regex-filter", {"regex": pattern})])
    assert e.value.args[0].endswith(text + "\n\nSmartModule Init Error: \n")


# version-uncertain code points (fsg_u_newer): U+1FAE8 and U+1E030 (assigned in
# Unicode 15), U+0295 (Ll -> Lo in Unicode 14)
NEWER = ["\U0001FAE8", "\U0001E030", "\u0295"]


@pytest.mark.parametrize("pattern", [r"\w", r"\d+", r"\p{Ll}", r"\p{Greek}", r"(?i)a", r"\bx", r"[^\W]"])
def test_version_uncertain_code_points_unsupported(pattern):
    """A pattern built from version-dependent tables (\\d \\w \\p, (?i) folding,
    Unicode \\b) meeting a code point whose class membership differs between
    this build's tables and regex-syntax 0.6.27 / 0.7.1's (Unicode 14 / 15) is
    FSG_E_UNSUPPORTED on both sides, match or not; other values are decided."""
    for cp in NEWER:
        t = ("x1 " + cp + " y").encode()
        with pytest.raises(ValueError) as e:
            dfa_match(pattern, t)
        assert e.value.args[0] == _ffi.FSG_E_UNSUPPORTED, (pattern, cp)
        with pytest.raises(ValueError):
            O.regex_is_match(pattern, t)
    t = "x1 é ω y".encode()
    assert dfa_match(pattern, t)[0] == O.regex_is_match(pattern, t)


@pytest.mark.parametrize("pattern", [r"a", r".", r"[^a]", r"\s", r"é+", r"\p{ASCII}", r"x\U0001FAE8", r"[\x{1FA00}-\x{1FAFF}]"])
def test_table_free_patterns_decide_newer_code_points(pattern):
    """Literals, '.', negated literal classes, White_Space and ASCII need no
    versioned table: values with newer code points are decided as usual."""
    for cp in NEWER:
        t = ("x " + cp).encode()
        assert dfa_match(pattern, t)[0] == O.regex_is_match(pattern, t), (pattern, cp)
