"""Generators of JSON record values for the JSON-field filter tests: valid
StructuredLog documents with extra fields, and byte-level mutations of them."""
import json
import random

LEVELS = ["debug", "info", "warn", "error"]
ESCAPES = ['\\n', '\\t', '\\"', '\\\\', '\\/', '\\u0041', '\\u00e9', '\\ud83d\\ude00', '\\b', '\\f', '\\r']


def rand_str(rng, n=8, escapes=True):
    out = []
    for _ in range(rng.randrange(n + 1)):
        if escapes and rng.random() < 0.1:
            out.append(rng.choice(ESCAPES))
        else:
            out.append(rng.choice("abcdefghij klmnopqrstuvwxyz0123456789-_:,{}[]"))
    return '"' + "".join(out) + '"'


def rand_value(rng, depth=0):
    r = rng.random()
    if depth > 3 or r < 0.35:
        return rng.choice([rand_str(rng), str(rng.randrange(-10**6, 10**6)), "true", "false", "null",
                           f"{rng.randrange(1000)}.{rng.randrange(1000)}", f"{rng.randrange(9)}e{rng.randrange(-5, 5)}",
                           "0", "-0", "18446744073709551615", "18446744073709551616"])
    if r < 0.65:
        return "[" + ",".join(rand_value(rng, depth + 1) for _ in range(rng.randrange(4))) + "]"
    return "{" + ",".join(f"{rand_str(rng, escapes=False)}:{rand_value(rng, depth + 1)}"
                          for _ in range(rng.randrange(4))) + "}"


def ws(rng):
    return rng.choice(["", "", "", " ", "\n", " \t", "\r\n "])


def valid_doc(rng):
    """A StructuredLog document (object or 2-element array form)."""
    level = rng.choice(LEVELS)
    lv = f'"{level}"' if rng.random() < 0.9 else '{' + ws(rng) + f'"{level}"' + ws(rng) + ':' + ws(rng) + 'null' + ws(rng) + '}'
    msg = rand_str(rng, 30)
    if rng.random() < 0.05:
        return f"{ws(rng)}[{ws(rng)}{lv}{ws(rng)},{ws(rng)}{msg}{ws(rng)}]{ws(rng)}"
    fields = [("level", lv), ("message", msg)]
    for _ in range(rng.randrange(4)):
        fields.append((json.loads(rand_str(rng, escapes=False)), rand_value(rng)))
    rng.shuffle(fields)
    body = ",".join(f"{ws(rng)}{json.dumps(k)}{ws(rng)}:{ws(rng)}{v}{ws(rng)}" for k, v in fields)
    return ws(rng) + "{" + body + "}" + ws(rng)


def mutate(rng, doc: str) -> bytes:
    b = bytearray(doc.encode())
    for _ in range(rng.randrange(1, 3)):
        op = rng.random()
        pos = rng.randrange(len(b) + 1)
        if op < 0.3 and len(b):
            del b[min(pos, len(b) - 1)]
        elif op < 0.6:
            b[pos:pos] = rng.choice([b'"', b',', b'}', b']', b'{', b'[', b':', b'\\', b'x', b'1', b'.', b'e', b'-',
                                     b' ', b'\x01', b'"level"', b'"message"', b'null', b'tru'])
        elif len(b):
            b[min(pos, len(b) - 1)] = rng.choice(b'",:{}[]\\ aZ09.-e\x00\x1f')
    return bytes(b)


def corpus(seed: int, n_valid: int, n_mut: int):
    rng = random.Random(seed)
    docs = [valid_doc(rng).encode() for _ in range(n_valid)]
    base = [valid_doc(rng) for _ in range(max(1, n_mut // 4))]
    docs += [mutate(rng, rng.choice(base)) for _ in range(n_mut)]
    fixed = [b"", b" ", b"{}", b"[]", b"null", b"5", b"-7", b"true", b'"x"', b'{"level":"info"}',
             b'{"message":"m"}', b'{"level":"info","level":"warn","message":"m"}', b'["warn"]',
             b'["warn","m","x"]', b'["warn","m",]', b'{"level":"INFO","message":"m"}',
             b'{"level":{"warn":5},"message":"m"}', b'{"level":{"warn":null,"x":1},"message":"m"}',
             b'{"level":{5:null},"message":"m"}', b'{"level":{"nope":null},"message":"m"}',
             b'{"level":"info","message":5}', b'{"level":"info","message":-12}', b'{"level":"info","message":[1]}',
             b'{"level":"info","message":{}}', b'{"level":"info","message":true}', b'{"level":"info","message":null}',
             b'{"level":"info","message":"\\ud800"}', b'{"level":"info","message":"\\udc00"}',
             b'{"level":"info","message":"\\ud800\\u0041"}', b'{"level":"info","message":"\\ud800x"}',
             b'{"level":"info","message":"a\\q"}', b'{"level":"info","message":"\\u12"}',
             b'{"level":"info","message":"x","n":01}', b'{"level":"info","message":"x","n":1.}',
             b'{"level":"info","message":"x","n":-}', b'{"level":"info","message":"x","n":1e+}',
             b'{"level":"info","message":"x","t":tru}', b'{"level":"info","message":"x","t":nul',
             b'{"level":"info","message":"x"} x', b'{"level":"info","message":"x",}', b'{,}',
             b'{"level":"info" "message":"x"}', b'{"level" "info","message":"x"}', b'{level:1}',
             b'{"lev\\u0065l":"warn","message":"m"}', b'{"level":"w\\u0061rn","message":"m"}',
             b'{"level":"warn","mess\\u0061ge":"m"}', b'{"level":"error","message":"caf\xc3\xa9"}',
             b'{"level":"error","message":"\xff"}', b'{"level":"error","x":"\xff","message":"m"}',
             b'{"level":"error","message":"a\x01"}', b'{"level":"error","x":"a\x01","message":"m"}',
             b'{"level":"info","message":"x","deep":' + b"[" * 70 + b"]" * 70 + b"}",
             b'{"level":"info","message":"x","deep":' + b"[" * 63 + b"]" * 63 + b"}",
             b'"\\u00e9"', b'"a\\"b"', b'"tab\\there"', b'1.5', b'-0', b'123456789012345678901',
             b'{"level":"debug","message":"x"}\n', b'\n\n  {"level"\n:\n"info"}',
             b'{"level":"info","message":"x","a":[1,2,{"b":[true,false,null,"s",-1.5e-3]}]}']
    return fixed + docs


# ---------------------------------------------------------------------------
# array_map_json_array inputs: JSON arrays of values
# ---------------------------------------------------------------------------
def am_value(rng, depth=0, sorted_keys=True, ints_only=True):
    """A JSON value.  ints_only: integers within u64/i64 (serde_json keeps them
    exact); sorted_keys: objects with strictly increasing keys (BTreeMap order)."""
    r = rng.random()
    if depth > 3 or r < 0.45:
        nums = [str(rng.randrange(-10**6, 10**6)), "0", "18446744073709551615", "-9223372036854775808"]
        if not ints_only:
            nums += [f"{rng.randrange(1000)}.{rng.randrange(1000)}", "-0", "18446744073709551616", "1e3",
                     f"{rng.randrange(-99, 99)}.{rng.randrange(10**6)}e{rng.randrange(-330, 310)}", "-2.5E-4",
                     "1e308", "4.9e-324", "0.1", "-0.0", "123456789012345678901234.5e-10", "1e16", "0.00001",
                     repr(rng.uniform(-1e6, 1e6)), "1e400" if rng.random() < 0.05 else "2.0"]
        return rng.choice([rand_str(rng), rand_str(rng, 3, False), rng.choice(nums), "true", "false", "null",
                           '"\\u001f\\u0001\\u007F"', '"caf\\u00e9 \\ud83d\\ude00"', '"\\/\\b"', '"ü\x7f"'])
    if r < 0.75:
        return "[" + ",".join(ws(rng) + am_value(rng, depth + 1, sorted_keys, ints_only) + ws(rng)
                              for _ in range(rng.randrange(4))) + "]"
    keys = list({json.loads(rand_str(rng, 4, escapes=False)) for _ in range(rng.randrange(4))})
    keys.sort(key=lambda k: k.encode())
    if not sorted_keys and len(keys) > 1:
        rng.shuffle(keys)
        if rng.random() < 0.3:
            keys.append(keys[0])
    return "{" + ",".join(f"{ws(rng)}{json.dumps(k)}{ws(rng)}:{ws(rng)}{am_value(rng, depth + 1, sorted_keys, ints_only)}"
                          for k in keys) + "}"


def array_doc(rng, sorted_keys=True, ints_only=True):
    n = rng.randrange(0, 12)
    return ws(rng) + "[" + ",".join(ws(rng) + am_value(rng, 0, sorted_keys, ints_only) + ws(rng)
                                    for _ in range(n)) + "]" + ws(rng)


ARRAY_FIXED = [b"[]", b" [ ] ", b"[1]", b'["Apple","Banana","Cranberry"]', b"[0,1,2,3,4,5,6,7,8,9]",
               b"[[[]]]", b'[{"a":1,"b":[2,{"c":null}]}]', b'["\\u0041\\/x"]', b'["\\u001F"]',
               b'[true,false,null]', b"[-0]", b"[1.5]", b"[1e2]", b"[18446744073709551616]",
               b"", b" ", b"{}", b'{"a":1}', b"5", b'"s"', b"null", b"[1,]", b"[,1]", b"[1 2]", b"[",
               b"[1", b'["a', b'["\\x"]', b'["\\ud800"]', b'["\\udc00"]', b'["a\x01"]', b'["\xff"]',
               b'["\xc3\xa9"]', b"[tru]", b"[nul", b"[01]", b"[1.]", b"[-]", b"[1e+]", b"[] x", b"[]]",
               b'[{"a" 1}]', b'[{1:2}]', b'[{"a":1,}]', b'[{"a":1 "b":2}]', b'[{"a":1}', b"[" * 130 + b"]" * 130,
               b"[" * 127 + b"]" * 127, b"[" * 128 + b"]" * 128, b'[{"b":1,"a":2}]', b'[{"a":1,"a":2}]',
               b'[{"\\u0061":1,"b":2}]', b'[\n1\n,\n"x"\n]', b'["\\ud83d\\ude00","\\"\\\\\\b\\f\\n\\r\\t"]']


def array_corpus(seed: int, n_valid: int, n_mut: int, sorted_keys=True, ints_only=True):
    rng = random.Random(seed)
    docs = [array_doc(rng, sorted_keys, ints_only).encode() for _ in range(n_valid)]
    base = [array_doc(rng, sorted_keys, ints_only) for _ in range(max(1, n_mut // 4))]
    docs += [mutate(rng, rng.choice(base)) for _ in range(n_mut)]
    return docs
