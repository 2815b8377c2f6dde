"""The committed fixtures are reproducible: every prime in primes.json is
produced by tests/golden/make_golden.py (the reference-case PRIMES plus the
repo-only EXTRA_PRIMES), with no hand-added entries.  The full regeneration
(`python tests/golden/make_golden.py`, which imports the reference) leaves the
fixture files byte-identical; this CPU test checks the part that needs no
reference: the prime table."""
import importlib.util
import json
import os

from conftest import ROOT

GOLDEN = os.path.join(ROOT, "tests", "golden")


def _generator():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_primes_json_is_generated():
    gen = _generator()
    want = {k: hex(v) for k, v in {**gen.PRIMES, **gen.EXTRA_PRIMES}.items()}
    got = json.load(open(os.path.join(GOLDEN, "primes.json")))
    assert got == want
    # the file is exactly what the generator writes
    assert open(os.path.join(GOLDEN, "primes.json")).read() == json.dumps(want, indent=1)
    for v in want.values():
        assert gen.is_probable_prime(int(v, 16))


def test_p256lo_is_the_smallest_256_bit_prime():
    gen = _generator()
    p = gen.EXTRA_PRIMES["p256lo"]
    assert p.bit_length() == 256
    assert all(not gen.is_probable_prime(x) for x in range((1 << 255) + 1, p, 2))
