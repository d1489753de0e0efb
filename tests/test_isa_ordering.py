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

STREAM_F64 = "_ZN8mireduce4kern13reduce_streamINS_5SumOpEddLi256ELi8ELb1ELi0EEEvNS0_4ArgsE"  # 256 x 8, hipcc schedule
DIRECT_F64_W8 = "_ZN8mireduce4kern13direct_kernelINS_5SumOpEdLi8EEEvPKNS_10DirectDescEmi"


def _disasm(tmp_path, obj: str, symbol: str, raw: bool = False) -> list:
    ensure_built()
    src = os.path.join(ROOT, "build", "obj", "kernels", obj)
    local = tmp_path / obj
    shutil.copy(src, local)
    subprocess.run([OBJDUMP, "--offloading", str(local)], check=True, capture_output=True, cwd=tmp_path)
    dev = [p for p in os.listdir(tmp_path) if p.startswith(obj) and p.endswith("gfx950")]
    assert dev, "no gfx950 code object in " + obj
    out = subprocess.run([OBJDUMP, "-d", f"--disassemble-symbols={symbol}", str(tmp_path / dev[0])], check=True,
                         capture_output=True, text=True).stdout
    lines = [ln for ln in out.splitlines() if ln.startswith("\t")]
    assert len(lines) > 100, f"{symbol} not found in {obj}"
    return lines if raw else [ln.split("//")[0].strip() for ln in lines]


def _first(ins, pattern, start=0):
    rx = re.compile(pattern)
    for i in range(start, len(ins)):
        if rx.search(ins[i]):
            return i
    return None


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


SMALL_F64 = "_ZN8mireduce4kern13reduce_streamINS_5SumOpEddLi256ELi4ELb1ELi0EEEvNS0_4ArgsE"  # <= 192 MB plan


def _max_in_flight(body: list) -> int:
    """Most 16-byte loads outstanding at once in a loop body that starts drained (vmcnt semantics)."""
    out, best = 0, 0
    for ln in body:
        if re.match(r"^(global|buffer)_load_dwordx4 ", ln):
            out += 1
            best = max(best, out)
        elif (m := re.match(r"^s_waitcnt vmcnt\((\d+)\)", ln)):
            out = min(out, int(m.group(1)))
    return best


def test_plain_body_keeps_its_loads_in_flight(tmp_path):
    # hipcc's schedule of the plain loop (the <= 192 MB default 256 x 4 x 3, e.g. the reference's
    # default 2^24 doubles; and 256 x 8): every tile's UNROLL independent 16-byte nt loads are in flight
    # together. Load scheduling moves this kernel by whole percents: hipcc once re-scheduled the
    # 512 x 16 body onto 60 VGPRs (7.3 -> 5.1 TB/s). (Until round 6 this test counted the longest run of
    # back-to-back loads anywhere in the 256 x 8 kernel — which was the contiguous split's loop, not the
    # interleaved one every default plan runs.)
    assert _vgpr_count(tmp_path, "reduce_tab_f64.o", STREAM_F64) >= 32
    for sym, unroll, want in ((SMALL_F64, 4, 4), (STREAM_F64, 8, 7)):
        lines = _disasm(tmp_path, "reduce_tab_f64.o", sym, raw=True)
        ins = [ln.split("//")[0].strip() for ln in lines]
        addr = [int(m.group(1), 16) if (m := re.search(r"// ([0-9A-F]+):", ln)) else None for ln in lines]
        loops = []
        for i, ln in enumerate(lines):  # loops with a tile's worth of loads
            t = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", ln)
            if t and ins[i].startswith("s_cbranch") and addr[i] and addr[0] + int(t.group(1), 16) < addr[i]:
                body = ins[addr.index(addr[0] + int(t.group(1), 16)):i + 1]
                if sum(bool(re.match(r"^global_load_dwordx4 .* nt$", x)) for x in body) == unroll:
                    loops.append(body)
        assert loops, sym
        assert max(_max_in_flight(b) for b in loops) >= want, (sym, [_max_in_flight(b) for b in loops])


HEADLINE_F64 = "_ZN8mireduce4kern13reduce_streamINS_5SumOpEddLi256ELi8ELb1ELi4EEEvNS0_4ArgsE"  # 8-byte > 192 MB


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


def _loops(lines: list) -> list:
    """The bodies (target .. backward branch) of the kernel's loops that issue >= 8 buffer loads."""
    addr = [int(m.group(1), 16) if (m := re.search(r"// ([0-9A-F]+):", ln)) else None for ln in lines]
    base = addr[0]
    ins = [ln.split("//")[0].strip() for ln in lines]
    out = []
    for i, ln in enumerate(lines):
        t = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", ln)
        if not (t and ins[i].startswith("s_cbranch") and addr[i] is not None and base + int(t.group(1), 16) < addr[i]):
            continue
        start = addr.index(base + int(t.group(1), 16))
        body = ins[start:i + 1]
        if sum(b.startswith("buffer_load") for b in body) >= 8:
            out.append(body)
    return out


def _norm(body: list) -> list:
    return [re.sub(r"\b[vs]\[?\d+(:\d+)?\]?|vcc_lo|vcc_hi|0x[0-9a-f]+|\b\d+\b", "R", x) for x in body]


def test_headline_hot_loop_unchanged_since_round5(tmp_path):
    # round 6 pruned the measured-null bodies (pipelined, strict window, contiguous /
    # balanced splits, ticketed fan-ins) from the production kernel; code the hot loop never runs has
    # moved hipcc's schedule of it before (104 -> 85 VGPRs, -1.5 %, docs/TUNING.md). The streaming loops
    # of the headline kernel must be instruction for instruction the ones BENCH_r05 measured
    # (tests/fixtures/headline_loop_r5.txt, registers and immediates normalised): same loads, same
    # waits, same interleave.
    with open(os.path.join(ROOT, "tests", "fixtures", "headline_loop_r5.txt")) as f:
        want = [blk.strip().splitlines() for blk in "".join(ln for ln in f if not ln.startswith("#")).split("--")]
    have = [_norm(b) for b in _loops(_disasm(tmp_path, "reduce_tab_f64.o", HEADLINE_F64, raw=True))]
    for w in want:
        assert w in have, "the headline kernel's streaming loop changed since round 5"
