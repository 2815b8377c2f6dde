"""End-to-end latency of the drop-in API on small inputs (MI355X): one
PySwizzle object, encode / gen_challenge / prove / verify of a BytesIO, best
and median of a few calls after a warm-up.  Experiment script (round 5).

--seed N: seeded primes, keys and challenges (A/B runs: the launch times
follow the longest rejection chain, i.e. the prime and the keys).
--only 1024: the PySwizzle-defaults case alone."""
import io
import json
import statistics
import sys
import time

sys.path.insert(0, ".")
from heartbeat_amd.PySwizzle import PySwizzle   # noqa: E402

_args = sys.argv[1:]
SEED = int(_args[_args.index("--seed") + 1]) if "--seed" in _args else None
ONLY = int(_args[_args.index("--only") + 1]) if "--only" in _args else None
if SEED is not None:
    import random
    _pys = sys.modules["heartbeat_amd.PySwizzle.PySwizzle"]
    _rng = random.Random(SEED)
    _pys._random_bytes = lambda n: bytes(_rng.getrandbits(8) for _ in range(n))

    def _seeded_prime(bits, _r=random.Random(SEED + 1)):
        while True:
            x = _r.getrandbits(bits) | (1 << (bits - 1)) | 1
            if _pys._is_probable_prime(x):
                return x
    _pys.getPrime = _seeded_prime


def timed(f, reps=7):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        r = f()
        ts.append((time.perf_counter() - t) * 1e3)
    return r, {"best_ms": round(min(ts), 3), "median_ms": round(statistics.median(ts), 3)}


out = {}
for label, S, bits, n in (("defaults S=10 1024-bit, 1 MiB", 10, 1024, 1 << 20),
                          ("S=16 256-bit, 1 MiB", 16, 256, 1 << 20),
                          ("S=16 256-bit, 64 MiB", 16, 256, 64 << 20)):
    if ONLY is not None and bits != ONLY:
        continue
    beat = PySwizzle(S, b"k" * 32, primebits=bits)
    data = bytes(bytearray((i * 2654435761 >> 13) & 0xFF for i in range(n)))
    f = io.BytesIO(data)

    def enc():
        f.seek(0)
        return beat.encode(f)

    (tag, state), te = timed(enc)
    chal, tc = timed(lambda: beat.gen_challenge(state))
    chal.chunks = min(chal.chunks, 10000)
    proof, tp = timed(lambda: beat.prove(f, chal, tag))
    ok, tv = timed(lambda: beat.verify(proof, chal, state))
    out[label] = {"encode": te, "gen_challenge": tc, "prove": tp, "verify": tv, "verified": ok,
                  "chunks": chal.chunks, "tags": len(tag.sigma)}
print(json.dumps(out, indent=1))
