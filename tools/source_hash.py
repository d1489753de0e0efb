#!/usr/bin/env python3
"""Build provenance: one hash of the native sources (``csrc/**``), embedded into the extension and
the apps at build time (``make`` -> build/gen/mireduce_source_hash.h -> csrc/runtime/version.cpp),
printed by ``bench.py`` / ``smoke()`` / ``reduction --version`` and compared with the working tree
by tests/test_provenance.py, so a stale prebuilt binary cannot produce a number unnoticed.

The hash is the first 16 hex digits of sha256 over git's index listing of ``csrc``: one line
``<mode> <blob sha1> 0\\t<path>\\n`` per file, sorted by path, i.e. exactly
``git ls-files -s csrc | sha256sum`` on a clean checkout — computed here from the files themselves,
so it needs no git (the GPU box has none) and covers files not yet committed.

    python tools/source_hash.py            # the hash
    python tools/source_hash.py --header   # a C header defining MIREDUCE_SOURCE_HASH
"""
from __future__ import annotations

import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_DIRS = {"__pycache__", ".git"}


def _files(root: str, sub: str = "csrc"):
    base = os.path.join(root, sub)
    for d, dirs, files in os.walk(base):
        dirs[:] = sorted(x for x in dirs if x not in SKIP_DIRS)
        for f in files:
            if f.endswith((".pyc", ".o", ".so", ".a")) or f.startswith("."):
                continue
            yield os.path.relpath(os.path.join(d, f), root).replace(os.sep, "/")


def listing(root: str = ROOT) -> str:
    lines = []
    for rel in sorted(_files(root)):
        p = os.path.join(root, rel)
        with open(p, "rb") as fh:
            data = fh.read()
        blob = hashlib.sha1(b"blob %d\0" % len(data) + data).hexdigest()
        mode = "100755" if os.access(p, os.X_OK) else "100644"
        lines.append(f"{mode} {blob} 0\t{rel}\n")
    return "".join(lines)


def source_hash(root: str = ROOT) -> str:
    return hashlib.sha256(listing(root).encode()).hexdigest()[:16]


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    h = source_hash()
    if "--header" in argv:
        print(f'#pragma once\n#define MIREDUCE_SOURCE_HASH "{h}"')
    else:
        print(h)
    return 0


if __name__ == "__main__":
    sys.exit(main())
