"""Pin the memory-ordering instruction sequences the single-pass / cross-rank / direct kernels rely
on. The kernels publish with relaxed atomics plus an explicit wait instead of a
full agent-scope release (which would write back the whole L2 on every arrival); that is correct
for the gfx950 ISA the compiler emits today, and these tests fail if a compiler change stops
emitting it. They read the gfx950 code object inside the built objects (CPU only: llvm-objdump)."""
import os
import re
import shutil
import subprocess

import pytest

from helpers import ROOT, ensure_built

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
pytestmark = pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not available")

STREAM_F64 = "_ZN8mireduce4kern13reduce_streamINS_5SumOpEddLi256ELi8ELb1ELb0ELi0EEEvNS0_4ArgsE"  # the >= 3 GB f64 plan
DIRECT_F64_W8 = "_ZN8mireduce4kern13direct_kernelINS_5SumOpEdLi8EEEvPKNS_10DirectDescEmi"


def _disasm(tmp_path, obj: str, symbol: str) -> list:
    ensure_built()
    src = os.path.join(ROOT, "build", "obj", "kernels", obj)
    local = tmp_path / obj
    shutil.copy(src, local)
    subprocess.run([OBJDUMP, "--offloading", str(local)], check=True, capture_output=True, cwd=tmp_path)
    dev = [p for p in os.listdir(tmp_path) if p.startswith(obj) and p.endswith("gfx950")]
    assert dev, "no gfx950 code object in " + obj
    out = subprocess.run([OBJDUMP, "-d", f"--disassemble-symbols={symbol}", str(tmp_path / dev[0])], check=True,
                         capture_output=True, text=True).stdout
    ins = [ln.split("//")[0].strip() for ln in out.splitlines() if ln.startswith("\t")]
    assert len(ins) > 100, f"{symbol} not found in {obj}"
    return ins


def _first(ins, pattern, start=0):
    rx = re.compile(pattern)
    for i in range(start, len(ins)):
        if rx.search(ins[i]):
            return i
    return None


def test_ticketed_fanin_publish_then_ticket_then_consume(tmp_path):
    # MIREDUCE_FANIN=flat|tree: partial stored write-through (sc1), drained, THEN the returning
    # ticket; after the barrier that broadcasts is_last, partials are read L1-bypassing (sc1).
    ins = _disasm(tmp_path, "reduce_tab_f64.o", STREAM_F64)
    ok = False
    for i, ln in enumerate(ins):
        if not re.search(r"^global_store_dwordx2 .* sc1$", ln):
            continue
        atom = _first(ins, r"^global_atomic_add .* sc0", i)
        if atom is None:
            continue
        wait = _first(ins, r"^s_waitcnt vmcnt\(0\)", i)
        bar = _first(ins, r"^s_barrier", atom)
        ld = _first(ins, r"^global_load_dwordx2 .* sc1$", bar or atom)
        if wait is not None and wait < atom and bar is not None and ld is not None:
            ok = True
            break
    assert ok, "no publish -> drain -> ticket -> barrier -> sc1-load sequence in the ticketed fan-in"


def test_polled_fanin_epoch_tagged_slots(tmp_path):
    # default fan-in: the launch's epoch (Workspace fan[0]) is loaded L2-bypassing
    # in the prologue and NOT waited for before the streaming body issues its first loads (its
    # latency hides under them); every workgroup stores two epoch-tagged 8-byte words (no drain, no
    # ticket); the finisher reads the sticky-error word (fan[1], offset:4), polls both words of a
    # slot (sc1 loads) with a bounded, sleeping loop, and finally stores the new epoch (a dword sc1
    # store back to fan[0]) — no slot is cleared.
    ins = _disasm(tmp_path, "reduce_tab_f64.o", STREAM_F64)
    ep = _first(ins, r"^global_load_dword v\d+, v\d+, (s\[\d+:\d+\]) sc1$")
    assert ep is not None and ep < 60, "epoch load is not in the prologue"
    fan = re.search(r"(s\[\d+:\d+\]) sc1$", ins[ep]).group(1)
    body = _first(ins, r"^global_load_dwordx4 .* nt$", ep)
    wait0 = _first(ins, r"^s_waitcnt vmcnt\(0\)", ep)
    assert body is not None and (wait0 is None or body < wait0), "a wait separates the epoch load from the body"
    st = _first(ins, r"^global_store_dwordx2 .* sc1$")
    assert st is not None and _first(ins, r"^global_store_dwordx2 .* offset:8 sc1$", st) is not None
    err = _first(ins, r"^global_load_dword v\d+, v\d+, " + re.escape(fan) + r" offset:4 sc1$", st)
    assert err is not None, "finisher does not read the sticky error word"
    poll = _first(ins, r"^global_load_dwordx2 .* sc1$", st)
    assert poll is not None and re.search(r"^global_load_dwordx2 .* offset:8 sc1$", ins[poll + 1])
    assert _first(ins, r"^s_sleep", poll) is not None and _first(ins, r"^s_memrealtime", st) is not None
    assert _first(ins, r"^global_store_dword v\d+, v\d+, " + re.escape(fan) + r" sc1$", poll) is not None, \
        "finisher does not advance the epoch"
    # (hipcc lays the polled and ticketed branches out in either order, so no check here compares
    # positions across the two branches)


def test_xrank_exchange_is_system_scope(tmp_path):
    ins = _disasm(tmp_path, "reduce_tab_f64.o", STREAM_F64)
    # fused cross-rank finish: mailbox words stored and polled at system scope (sc0 sc1), bounded
    st = _first(ins, r"^flat_store_dwordx2 .* sc0 sc1$")
    ld = _first(ins, r"^flat_load_dwordx2 .* sc0 sc1$", st or 0)
    assert st is not None and ld is not None and st < ld
    assert _first(ins, r"^s_sleep", ld) is not None
    assert _first(ins, r"^s_memrealtime", st) is not None, "the poll is no longer time-bounded"


def test_direct_barrier_release_and_acquire(tmp_path):
    ins = _disasm(tmp_path, "direct.o", DIRECT_F64_W8)
    wb = _first(ins, r"^buffer_wbl2 sc0 sc1")  # system-scope release before raising a flag
    flag = _first(ins, r"^flat_store_dword .* sc0 sc1$", wb or 0)
    poll = _first(ins, r"^flat_load_dword .* sc0 sc1$", flag or 0)
    inv = _first(ins, r"^buffer_inv sc0 sc1", poll or 0)  # system-scope acquire after the wait
    assert None not in (wb, flag, poll, inv) and wb < flag < poll < inv


def _vgpr_count(tmp_path, obj: str, symbol: str) -> int:
    ensure_built()
    local = tmp_path / obj
    shutil.copy(os.path.join(ROOT, "build", "obj", "kernels", obj), local)
    subprocess.run([OBJDUMP, "--offloading", str(local)], check=True, capture_output=True, cwd=tmp_path)
    dev = [p for p in os.listdir(tmp_path) if p.startswith(obj) and p.endswith("gfx950")][0]
    readelf = os.path.join(os.path.dirname(OBJDUMP), "llvm-readelf")
    notes = subprocess.run([readelf, "--notes", str(tmp_path / dev)], check=True, capture_output=True,
                           text=True).stdout
    # amdhsa.kernels metadata: ".name: <sym>" followed (within the same entry) by ".vgpr_count: N"
    m = re.search(r"\.name:\s+" + re.escape(symbol) + r"\s*\n(?:.*\n){0,40}?\s+\.vgpr_count:\s+(\d+)", notes)
    assert m, f"no metadata for {symbol}"
    return int(m.group(1))


def test_headline_kernel_keeps_its_loads_in_flight(tmp_path):
    # 256 x 8 f64 (the >= 3 GB plan): the streaming loop issues its 8 independent 16-byte nt loads
    # back to back before the first wait (>= 32 VGPRs of data). Load scheduling moves this kernel
    # by whole percents: hipcc once re-scheduled the 512 x 16 body onto 60 VGPRs (7.3 -> 5.1 TB/s),
    # and today's 512 x 16 body keeps only ~9 of its 16 loads in flight.
    assert _vgpr_count(tmp_path, "reduce_tab_f64.o", STREAM_F64) >= 32
    ins = _disasm(tmp_path, "reduce_tab_f64.o", STREAM_F64)
    run, best = 0, 0
    for ln in ins:
        if re.match(r"^global_load_dwordx4 .* nt$", ln):
            run += 1
            best = max(best, run)
        elif ln.startswith("s_waitcnt") or ln.startswith("v_add_f64"):
            run = 0
    assert best >= 8, best


HEADLINE_F64 = "_ZN8mireduce4kern13reduce_streamINS_5SumOpEddLi256ELi8ELb1ELb0ELi4EEEvNS0_4ArgsE"  # 8-byte > 192 MB


def test_headline_kernel_explicit_load_window(tmp_path):
    # The tuned plan for 8-byte arrays above 192 MB (the 1e9-double headline and the 1 GB N=8 shard):
    # 256 x 8 with an explicit load window of 4 (reduce_kernels.hpp stream_window; profiles/r3_window).
    # Its streaming loop is raw buffer loads that keep the nt bit (a plain-pointer nontemporal load
    # lost it under this interleave) in the pinned order "issue, wait until 4 remain, consume":
    # 8 x (buffer_load nt, s_waitcnt vmcnt(4), 2 x v_add_f64) per tile, no waterfall around them.
    ins = _disasm(tmp_path, "reduce_tab_f64.o", HEADLINE_F64)
    seq = []
    for ln in ins:
        if ln.startswith("buffer_load_dwordx4"):
            seq.append("B" if ln.endswith(" nt") else "Bplain")
        elif ln.startswith("global_load_dwordx4"):
            seq.append("G")
        elif ln.startswith("s_waitcnt vmcnt"):
            seq.append("W" + re.search(r"vmcnt\((\d+)\)", ln).group(1))
        elif ln.startswith("v_add_f64"):
            seq.append("a")
        elif ln.startswith("s_and_saveexec"):
            seq.append("X")
    s = " ".join(seq)
    assert "Bplain" not in s, "a streaming buffer load lost its nt bit"
    assert " ".join(["B W4 a a"] * 8) in s, s[:300]
    # the fan-in epoch load sits in the prologue and no vmcnt(0) separates it from the first body load
    ep = _first(ins, r"^global_load_dword v\d+, v\d+, s\[\d+:\d+\] sc1$")
    body = _first(ins, r"^buffer_load_dwordx4 .* nt$")
    assert ep is not None and body is not None and ep < body
    assert _first(ins, r"^s_waitcnt vmcnt\(0\)", ep) is None or _first(ins, r"^s_waitcnt vmcnt\(0\)", ep) > body
