// Build provenance: the hash of the native sources this binary was built from (tools/source_hash.py:
// sha256 of `git ls-files -s csrc`, first 16 hex digits, computed at build time by the Makefile).
// bench.py, smoke(), `reduction --version` and the JSON sidecars report it; tests/test_provenance.py
// compares it with the working tree, so a stale prebuilt binary cannot produce a number unnoticed.
#pragma once

namespace mireduce {

const char* source_hash();

}  // namespace mireduce
