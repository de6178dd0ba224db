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
            r"(?i)[[:lower:]]{2}\b"]
WORD = ("\\b", "\\B", "\\w", "\\W")


def texts(rng):
    alpha = "abcdxyzABCD0123456789- \t\n.é☺αβω"
    out = ["", "a", "abc", "ac", "xxy", "123-45-6789", "my ssn 987-65-4321!", "colour  x", "☺A", "aé",
           "abcd", "cd", "ab", "timeouts", "αβγ", "aaa", "abcbcd"]
    for _ in range(60):
        out.append("".join(rng.choice(alpha) for _ in range(rng.randint(0, 24))))
    return out


@pytest.mark.parametrize("pattern", PATTERNS)
def test_dfa_matches_oracle(pattern):
    rng = random.Random(hash(pattern) & 0xFFFF)
    word = any(w in pattern for w in WORD)
    for t in texts(rng):
        b = t.encode()
        if word and not b.isascii():  # Unicode word semantics: the kernel reports UNSUPPORTED
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
                                      ("(?m)^a", _ffi.FSG_E_UNSUPPORTED), ("(?x)a b", _ffi.FSG_E_UNSUPPORTED),
                                      (r"\pL", _ffi.FSG_E_UNSUPPORTED), ("(?i)é", _ffi.FSG_E_UNSUPPORTED),
                                      ("[[a]]", _ffi.FSG_E_UNSUPPORTED)])
def test_errors_agree_with_oracle(bad, code):
    with pytest.raises(ValueError) as e:
        dfa_match(bad, b"x")
    assert e.value.args[0] == code
    with pytest.raises(ValueError):
        O.regex_is_match(bad, b"x")
