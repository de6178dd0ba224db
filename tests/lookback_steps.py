"""Driver for the look_back known answers (tests/golden/kats.json "look_back"):
one chain per "new_chain" step, look_back over the records the SPU would read
from the replica, process of one input.  Shared by the oracle test (CPU) and
the GPU parity test, so both are checked against the same reference vectors."""


def run_lookback_case(case, new_chain, look_back, process):
    """new_chain(lookback) -> chain; look_back(chain, values) -> (error dict | None,
    invocations); process(chain, values) -> (values, invocations)."""
    chain = new_chain(case["lookback"])
    inv = 0
    for step in case["steps"]:
        if "new_chain" in step:
            chain = new_chain(step["new_chain"])
            inv = 0
        elif "look_back" in step:
            err, n = look_back(chain, step["look_back"])
            inv += n
            exp = step.get("error")
            if exp is None:
                assert err is None, (case["name"], err)
            else:
                assert err is not None, case["name"]
                assert err["hint"] == exp["hint"]
                assert err["offset"] == exp["offset"]
                assert err["key"] == (exp["key"].encode() if exp["key"] is not None else None)
                assert err["value"] == exp["value"].encode()
        else:
            vals, n = process(chain, step["process"])
            inv += n
            assert vals == [v.encode() for v in step["expect"]], (case["name"], step)
    if "invocation_count" in case:
        assert inv == case["invocation_count"], case["name"]
