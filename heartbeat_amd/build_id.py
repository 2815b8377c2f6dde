"""Provenance of libhbswizzle.so: content hashes of the sources it is built from.

The Makefile (csrc/Makefile) compiles ``hb_build_id()`` = SHA-256 of
``sources_digest()`` + "|" + the compiler flags into the library, and keys
every object file on a stamp holding the hash of that object's own inputs, so
objects restored from another tree state cannot satisfy make.  ``_native.lib()``
recomputes the digest from the tree next to the library and refuses a library
built from other sources (a touched but unchanged tree still matches: the hash
is over contents, not times).

Command line (used by the Makefile):
  python3 build_id.py digest FILE...      SHA-256 over the named files (+ $HB_ID_FLAGS)
  python3 build_id.py id                  the library id for $HB_ID_FLAGS
  python3 build_id.py stamp PATH VALUE    write VALUE to PATH unless it already holds it
  python3 build_id.py stamp-digest PATH FILE...   stamp PATH with the digest of FILE...
"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SUFFIXES = (".hip", ".hpp", ".cpp", ".h")


def source_files(root=None):
    """(relative name, path) of every input of libhbswizzle.so, sorted:
    heartbeat_amd/csrc/{*.hip,*.hpp,*.cpp,*.h,Makefile} and include/hbswizzle.h."""
    root = os.path.dirname(HERE) if root is None else root
    csrc = os.path.join(root, "heartbeat_amd", "csrc")
    out = []
    for name in sorted(os.listdir(csrc)):
        p = os.path.join(csrc, name)
        if os.path.isfile(p) and (name.endswith(SUFFIXES) or name == "Makefile"):
            out.append(("heartbeat_amd/csrc/" + name, p))
    out.append(("include/hbswizzle.h", os.path.join(root, "include", "hbswizzle.h")))
    return out


def digest_files(named):
    h = hashlib.sha256()
    for rel, path in named:
        with open(path, "rb") as fh:
            data = fh.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()


def sources_digest(root=None):
    return digest_files(source_files(root))


def library_id(digest, flags):
    """hb_build_id() of a library built from sources with `digest` and `flags`."""
    return hashlib.sha256((digest + "|" + " ".join(flags.split())).encode()).hexdigest()


def main(argv):
    flags = os.environ.get("HB_ID_FLAGS", "")
    if argv[:1] == ["digest"]:
        named = [(os.path.basename(p), p) for p in argv[1:]]
        print(library_id(digest_files(named), flags))
    elif argv[:1] == ["id"]:
        print(library_id(sources_digest(), flags))
    elif argv[:1] in (["stamp"], ["stamp-digest"]) and len(argv) >= 3:
        path = argv[1]
        if argv[0] == "stamp-digest":
            value = library_id(digest_files([(os.path.basename(p), p) for p in argv[2:]]), flags)
        elif len(argv) == 3:
            value = argv[2]
        else:
            sys.stderr.write(__doc__)
            return 2
        try:
            with open(path) as fh:
                if fh.read().strip() == value:
                    return 0
        except OSError:
            pass
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as fh:
            fh.write(value + "\n")
    else:
        sys.stderr.write(__doc__)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
