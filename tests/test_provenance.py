"""Build provenance: the native binaries carry the hash of the csrc tree they were
built from (tools/source_hash.py = sha256 of `git ls-files -s csrc`), and it must equal the working
tree's — a stale prebuilt extension or app (they travel to the GPU box with every gpurun snapshot)
cannot produce a number unnoticed. CPU only."""
import os
import subprocess
import sys

from helpers import BIN, ROOT, ensure_built

sys.path.insert(0, os.path.join(ROOT, "tools"))
import source_hash  # noqa: E402


def test_extension_hash_equals_working_tree():
    ensure_built()
    from cuda_mpi_reductions_amd._native import native
    assert native().source_hash() == source_hash.source_hash()


def test_apps_report_the_same_hash():
    ensure_built()
    h = source_hash.source_hash()
    for app in ("reduction", "reduce_xgmi", "reduce_mpi", "bandwidth_test"):
        r = subprocess.run([os.path.join(BIN, app), "--version"], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0 and f"native source {h}" in r.stdout, (app, r.stdout, r.stderr)


def test_listing_matches_git_index_format(tmp_path):
    # one "<mode> <blob sha1> 0\t<path>" line per file, exactly git's index listing
    d = tmp_path / "csrc" / "x"
    d.mkdir(parents=True)
    (d / "a.cpp").write_bytes(b"int a;\n")
    lst = source_hash.listing(str(tmp_path))
    blob = subprocess.run(["git", "hash-object", str(d / "a.cpp")], capture_output=True, text=True).stdout.strip()
    assert lst == f"100644 {blob} 0\tcsrc/x/a.cpp\n"
    if subprocess.run(["git", "-C", ROOT, "rev-parse"], capture_output=True).returncode == 0:
        clean = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "csrc"], capture_output=True,
                               text=True).stdout.strip() == ""
        if clean:  # a clean checkout: the hash IS sha256(git ls-files -s csrc)
            import hashlib
            ls = subprocess.run(["git", "-C", ROOT, "ls-files", "-s", "csrc"], capture_output=True,
                                text=True).stdout
            assert hashlib.sha256(ls.encode()).hexdigest()[:16] == source_hash.source_hash()
