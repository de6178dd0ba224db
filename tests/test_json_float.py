"""JSON floats: serde_json 1.0.96's f64 reading (f64_from_parts, the default
build without float_roundtrip), ryu's format (Value::to_string) and Rust's
Display behind serde's WithDecimalPoint ("invalid type: floating point `..`").

Three independent statements are compared: the product's host+device header
(fluvio_amd/csrc/fsg_float.h, through the host-only debug library), the oracle
(oracle/fsg_json.c: glibc printf/strtod shortest search), and the Python model
below (serde's reader rewritten over Python floats; shortest digits from
Python's repr, which is David Gay's shortest round-trip).  No reference test
holds float vectors: parity unpinned beyond this agreement, noted in DESIGN.md."""
import ctypes
import decimal
from fractions import Fraction
import random
import struct

import pytest

from fluvio_amd import _ffi
from oracle import oracle as O

POW10 = [float("1e%d" % k) for k in range(309)]


def serde_read(t: str):
    """de.rs parse_integer .. f64_from_parts: ("int", text) / ("f64", value) / ("range", index)."""
    i, n = 0, len(t)
    pos = t[0] != "-"
    if not pos:
        i = 1
    sig, exp, flt = 0, 0, False
    U = (1 << 64) - 1

    def over(s, d):
        return s > U // 10 or (s == U // 10 and d > U % 10)
    if t[i] == "0":
        i += 1
    else:
        while i < n and t[i].isdigit():
            d = int(t[i])
            if over(sig, d):
                flt = True
                while i < n and t[i].isdigit():
                    i += 1
                    exp += 1
                break
            sig = sig * 10 + d
            i += 1
    if i < n and t[i] == ".":
        flt = True
        i += 1
        ov = False
        while i < n and t[i].isdigit():
            d = int(t[i])
            ov = ov or over(sig, d)
            if not ov:
                sig = sig * 10 + d
                exp -= 1
            i += 1
    if i < n and t[i] in "eE":
        flt = True
        i += 1
        pe = True
        if t[i] in "+-":
            pe = t[i] == "+"
            i += 1
        e = int(t[i])
        i += 1
        while i < n and t[i].isdigit():
            d = int(t[i])
            i += 1
            if e > 214748364 or (e == 214748364 and d > 7):
                if sig != 0 and pe:
                    return ("range", i)
                return ("f64", 0.0 if pos else -0.0)
            e = e * 10 + d
        exp = max(-2 ** 31, min(2 ** 31 - 1, exp + e if pe else exp - e))
    if not flt:
        if pos or 0 < sig <= 1 << 63:
            return ("int", t)
        return ("f64", -float(sig))
    f = float(sig)
    while True:
        if abs(exp) <= 308:
            if exp >= 0:
                f *= POW10[abs(exp)]
                if f == float("inf"):
                    return ("range", n)
            else:
                f /= POW10[abs(exp)]
            break
        if f == 0.0:
            break
        if exp >= 0:
            return ("range", n)
        f /= 1e308
        exp += 308
    return ("f64", f if pos else -f)


def digits(x):
    """shortest round-trip digits of |x| > 0 and k with |x| = 0.digits x 10^k"""
    tup = decimal.Decimal(repr(abs(x))).normalize().as_tuple()
    ds = "".join(map(str, tup.digits))
    return ds, len(ds) + tup.exponent


def ryu_py(x):
    if x == 0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    sg = "-" if x < 0 else ""
    ds, kk = digits(x)
    ln, e = len(ds), kk - len(ds)
    if e >= 0 and kk <= 16:
        return sg + ds + "0" * (kk - ln) + ".0"
    if 0 < kk <= 16:
        return sg + ds[:kk] + "." + ds[kk:]
    if -5 < kk <= 0:
        return sg + "0." + "0" * (-kk) + ds
    return sg + ds[0] + ("." + ds[1:] if ln > 1 else "") + "e" + str(kk - 1)


def display_py(x):
    """Rust Display + WithDecimalPoint.  Rust's shortest digits (flt2dec dragon
    format_shortest) round an exact tie upward where repr keeps the even digit."""
    sg = "-" if str(x).startswith("-") else ""
    if x == 0:
        return sg + "0.0"
    ds, kk = digits(x)
    unit = Fraction(10) ** (kk - len(ds))
    if Fraction(abs(x)) - int(ds) * unit == unit / 2:
        up = str(int(ds) + 1)
        if float(up + "e" + str(kk - len(ds))) == abs(x):
            ds, kk = up.rstrip("0"), kk + (len(up) - len(ds))
    if kk <= 0:
        s = "0." + "0" * (-kk) + ds
    elif kk < len(ds):
        s = ds[:kk] + "." + ds[kk:]
    else:
        s = ds + "0" * (kk - len(ds))
    return sg + s + ("" if "." in s else ".0")


def product(t: str):
    f = _ffi.debug_lib().fsg_debug_json_number
    b = t.encode()
    bits = ctypes.c_uint64()
    ry, dp = ctypes.create_string_buffer(400), ctypes.create_string_buffer(400)
    rl, dl, e = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    k = f(b, len(b), ctypes.byref(bits), ry, ctypes.byref(rl), dp, ctypes.byref(dl), ctypes.byref(e))
    if k == 0:
        return ("int", t)
    if k == 2:
        return ("range", e.value)
    x = struct.unpack("<d", struct.pack("<Q", bits.value))[0]
    return ("f64", x, ry.raw[:rl.value].decode(), dp.raw[:dl.value].decode())


def numbers(rng, count):
    out = ["0.1", "1e16", "1e15", "1.5e-7", "100.0", "-0", "-0.0", "5e-324", "2.2250738585072014e-308",
           "1.7976931348623157e308", "18446744073709551615", "18446744073709551616", "-9223372036854775808",
           "-9223372036854775809", "1e400", "-1e400", "1e-400", "0.000001", "0.00001", "1234.5", "-1.25e-5",
           "1e2147483647", "1e2147483648", "0e99999999999", "1e-99999999999", "123456789012345678901234567890",
           "1844674407370955161.9", "18446744073709551619.5e-3", "0.30000000000000004", "9007199254740993.0",
           "1E5", "1e+5", "1.0e-0", "4.9406564584124654e-324", "2.5", "0.5", "562949953421312.25"]
    for _ in range(count):
        r = rng.random()
        if r < 0.35:  # random finite doubles, shortest text
            x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(63)))[0]
            if x != x or x in (float("inf"),):
                continue
            out.append(repr(x if rng.random() < 0.5 else -x).replace("e+", "e"))
        elif r < 0.6:  # decimal strings of random length / exponent
            m = str(rng.randint(1, 10 ** rng.randint(1, 25)))
            p = rng.randint(0, len(m))
            s = m[:p] + ("." + m[p:] if p < len(m) else "")
            if s.startswith("."):
                s = "0" + s
            if rng.random() < 0.6:
                s += "e" + str(rng.randint(-340, 330))
            out.append(("-" if rng.random() < 0.3 else "") + s)
        elif r < 0.8:  # short human decimals
            out.append("%d.%0*d" % (rng.randint(0, 99999), rng.randint(1, 4), rng.randint(0, 999)))
        else:  # long integers
            out.append(str(rng.randint(0, 10 ** rng.randint(15, 30))))
    return out


def test_float_reader_and_formats_agree():
    rng = random.Random(11)
    n_f64 = 0
    for t in numbers(rng, 6000):
        want = serde_read(t)
        got = product(t)
        assert got[0] == want[0], (t, got, want)
        if want[0] == "range":
            assert got[1] == want[1], t
            continue
        if want[0] == "int":
            continue
        x = want[1]
        assert struct.pack("<d", got[1]) == struct.pack("<d", x), (t, got[1], x)
        assert got[2] == ryu_py(x), (t, got[2], ryu_py(x))
        assert got[3] == display_py(x), (t, got[3], display_py(x))
        # the oracle: array_map re-serializes the element with ryu
        st, els = O.json_array_map(("[" + t + "]").encode())
        assert st == "ok" and els == [got[2].encode()], (t, st, els)
        n_f64 += 1
    assert n_f64 > 3000


def test_float_messages_oracle():
    """"invalid type: floating point `..`" (serde Unexpected::Float + WithDecimalPoint)
    and "number out of range" with serde_json's positions."""
    assert O.json_structured_log(b'{"message": 1.5}')[1] == \
        "invalid type: floating point `1.5`, expected a string at line 1 column 15"
    assert O.json_structured_log(b'{"message": 1e2}')[1] == \
        "invalid type: floating point `100.0`, expected a string at line 1 column 15"
    assert O.json_structured_log(b'{"message": -0}')[1] == \
        "invalid type: floating point `-0.0`, expected a string at line 1 column 14"
    assert O.json_structured_log(b'{"message": 1e400}')[1] == "number out of range at line 1 column 17"
    assert O.json_structured_log(b'{"message": 1e99999999999}')[1] == "number out of range at line 1 column 24"
    assert O.json_structured_log(b'{"level": 1.5}')[1] == "expected value at line 1 column 11"  # deserialize_enum
    assert O.json_array_map(b"[1, 2e-7, -0, 3.25]") == ("ok", [b"1", b"2e-7", b"-0.0", b"3.25"])
    assert O.json_array_map(b'[{"b": 1.0, "a": [1e300]}]') == ("ok", [b'{"a":[1e300],"b":1.0}'])
