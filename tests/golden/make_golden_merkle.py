#!/usr/bin/env python3
"""Golden vectors for Merkle's KeyedPRF-positioned chunk hashing from the
REFERENCE (heartbeat/Merkle/Merkle.py:447-515, MerkleHelper).

Runs only in the build container (reads /root/reference).  Imports the
unmodified reference modules heartbeat/exc.py, heartbeat/util.py and the
heartbeat/Merkle package under a synthetic ``heartbeat`` package with the
offline PyCrypto-API shim (tests/golden/shim), as make_golden.py does, and
records MerkleHelper.get_next_seed / get_chunk_hash outputs.

Output: merkle_cases.json next to this script (inputs and outputs only).
"""
import hashlib
import importlib.util
import io
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "shim"))


def load_reference():
    pkg = types.ModuleType("heartbeat")
    pkg.__path__ = [os.path.join(REF, "heartbeat")]
    sys.modules["heartbeat"] = pkg

    def load(name, path, is_pkg=False):
        kw = {"submodule_search_locations": [os.path.dirname(path)]} if is_pkg else {}
        spec = importlib.util.spec_from_file_location(name, path, **kw)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    load("heartbeat.exc", os.path.join(REF, "heartbeat/exc.py"))
    load("heartbeat.util", os.path.join(REF, "heartbeat/util.py"))
    return load("heartbeat.Merkle", os.path.join(REF, "heartbeat/Merkle/__init__.py"), True)


def det_bytes(tag, n):
    out = b""
    i = 0
    while len(out) < n:
        out += hashlib.sha256(("%s/%d" % (tag, i)).encode()).digest()
        i += 1
    return out[:n]


def main():
    M = load_reference()
    H = M.MerkleHelper
    files = {
        "test.txt": open(os.path.join(HERE, "files", "test.txt"), "rb").read(),
        "test3.txt": open(os.path.join(HERE, "files", "test3.txt"), "rb").read(),
        "rand100k": det_bytes("merkle-file", 100003),
        "tiny5": det_bytes("merkle-tiny", 5),
    }
    cases = []
    key = det_bytes("merkle-key", 32)
    seed = det_bytes("merkle-seed", 32)
    chain = []
    s = seed
    for _ in range(40):
        s = H.get_next_seed(key, s)
        chain.append(s)
    for fname, data in files.items():
        for chunksz in (8192, 1, 100, 4096, len(data), len(data) + 10):
            seeds = chain[:16]
            leaves = [H.get_chunk_hash(io.BytesIO(data), sd, None, chunksz).hex() for sd in seeds]
            # explicit filesz (Merkle.prove passes tag.filesz) and a small bufsz
            leaves2 = [H.get_chunk_hash(io.BytesIO(data), sd, len(data), chunksz, 37).hex() for sd in seeds[:4]]
            cases.append({"file": fname, "chunksz": chunksz, "seeds": [x.hex() for x in seeds],
                          "leaves": leaves, "leaves_explicit_small_buf": leaves2})
    # 16- and 24-byte seeds (AES-128 / AES-192 KeyedPRF keys)
    for sl in (16, 24):
        seeds = [det_bytes("merkle-seed-%d-%d" % (sl, k), sl) for k in range(12)]
        data = files["rand100k"]
        leaves = [H.get_chunk_hash(io.BytesIO(data), sd, None, 8192).hex() for sd in seeds]
        cases.append({"file": "rand100k", "chunksz": 8192, "seeds": [x.hex() for x in seeds], "leaves": leaves})
    out = {"generator": "tests/golden/make_golden_merkle.py",
           "reference": "heartbeat/Merkle/Merkle.py:447-515 (MerkleHelper)",
           "chain": {"key": key.hex(), "seed": seed.hex(), "seeds": [x.hex() for x in chain]},
           "files": {k: {"len": len(v), "sha256": hashlib.sha256(v).hexdigest()} for k, v in files.items()},
           "cases": cases}
    with open(os.path.join(HERE, "merkle_cases.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote %d cases" % len(cases))


if __name__ == "__main__":
    main()
