"""Static checks on the gfx950 code object of the fast kernel (CPU only).

The fast kernel's latency hiding rests on properties the compiler can silently
break: no scratch spills (a reload waits vmcnt(0) and drains the LDS-DMA
look-ahead), few vmcnt(0) waits, and hand-written two-instruction scalar loads
whose first destination must not overlap the base the second one reads (that
overlap faulted on the GPU).  The code object is disassembled straight out of
the in-tree libusv.so.
"""
import os
import re
import shutil
import subprocess

import pytest

from unsynchronized_stereo_vision_proj325_amd import _lib

LLVM = "/opt/rocm/lib/llvm/bin"


def _disassembly(tmp_path):
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libusv.so not built")
    if not shutil.which("objcopy") or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("objcopy / llvm-objdump not available")
    fat = tmp_path / "fat.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", _lib.LIB_PATH, str(fat)],
                   check=True)
    # the section holds one offload bundle per translation unit: unbundle each one's gfx950 object
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = ""
    for n, a in enumerate(starts):
        b = starts[n + 1] if n + 1 < len(starts) else len(data)
        part, co = tmp_path / f"bundle{n}.bin", tmp_path / f"gfx950_{n}.co"
        part.write_bytes(data[a:b])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                       check=True)
        out += subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(co)], check=True,
                              capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur and line.startswith("\t"):
            code, _, comment = line.partition("//")
            a = re.match(r"\s*([0-9A-F]+):", comment)
            funcs[cur].append(Insn(code.strip(), int(a.group(1), 16) if a else -1))
    return funcs


class Insn(str):
    """An instruction's text (a str, so the simple checks compare text) plus its byte address."""

    def __new__(cls, text, addr):
        o = super().__new__(cls, text)
        o.addr = addr
        return o


def _sregs(tok):
    tok = tok.rstrip(",")
    m = re.match(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()


@pytest.fixture(scope="module")
def fast_kernels(tmp_path_factory):
    funcs = _disassembly(tmp_path_factory.mktemp("isa"))
    fast = {k: v for k, v in funcs.items()
            if "sad_fast_kernel" in k or "sad_pair_kernel" in k or "ssd_fast_kernel" in k or "sad_group_kernel" in k}
    assert sum("sad_fast_kernel" in k for k in fast) == 21, sorted(fast)  # r = 1..7 x NW = 1, 2, 4
    assert sum("sad_pair_kernel" in k for k in fast) == 6, sorted(fast)   # r = 5..7 x NW = 1, 2
    assert sum("ssd_fast_kernel" in k for k in fast) == 9, sorted(fast)   # r = 5..7 x NW = 1, 2, 4
    assert sum("sad_group_kernel" in k for k in fast) == 6, sorted(fast)  # r = 2..4 x G = 2, 4
    return fast


def test_no_scratch(fast_kernels):
    bad = {k: sum("scratch_" in i for i in v) for k, v in fast_kernels.items()}
    assert not any(bad.values()), {k: n for k, n in bad.items() if n}


def test_few_full_vmem_drains(fast_kernels):
    # allowed: kernel-entry LUT copy, the final drain and the exit paths per border variant
    counts = {k: sum(i.startswith("s_waitcnt") and "vmcnt(0)" in i for i in v) for k, v in fast_kernels.items()}
    assert all(n <= 8 for n in counts.values()), counts


def test_split_scalar_loads_do_not_clobber_their_base(fast_kernels):
    for name, ins in fast_kernels.items():
        for a, b in zip(ins, ins[1:]):
            # immediate-offset form (warm-up rows) and SGPR-offset form (steady rows)
            m1 = re.match(r"s_load_dwordx4 (\S+), (\S+), (?:0x0|s\d+)$", a)
            m2 = re.match(r"s_load_dword(?:x2)? (\S+), (\S+), (?:0x10|s\d+ offset:0x10)$", b)
            if m1 and m2 and m1.group(2) == m2.group(2):
                assert not (_sregs(m1.group(1)) & _sregs(m2.group(2))), (name, a, b)


def _successors(ins):
    at = {i.addr: k for k, i in enumerate(ins)}
    out = []
    for k, i in enumerate(ins):
        m = re.match(r"s_(c?)branch\w* (\d+)", i)
        if m:
            off = int(m.group(2))
            off = off - 65536 if off >= 32768 else off
            s = [at[i.addr + 4 + 4 * off]] if i.addr + 4 + 4 * off in at else []
            if m.group(1):
                s.append(k + 1)
        elif i.startswith(("s_endpgm", "s_setpc_b64")):
            s = []
        else:
            s = [k + 1]
        out.append([j for j in s if j < len(ins)])
    return out


def inflight_scalar_load_hazards(ins):
    """Instructions that touch an SGPR while a scalar load writing it may still be in flight.

    A scalar load writes its destination whenever its data returns; only
    s_waitcnt lgkmcnt(0) retires it (they return out of order).  The hand-written
    s_load of the next row's L words is invisible to the compiler's waitcnt
    pass, so on a path where that value is dead (the loop exit) the compiler may
    reuse the registers -- the late return then clobbered the flush's row count.
    Forward dataflow over the CFG: the set of in-flight SGPRs at each instruction.
    """
    succ = _successors(ins)
    state = [None] * len(ins)
    state[0] = frozenset()
    work, bad = [0], set()
    while work:
        k = work.pop()
        cur, i = set(state[k]), ins[k]
        toks = i.replace(",", " ").split()
        if i.startswith("s_waitcnt") and "lgkmcnt(0)" in i:
            cur = set()
        elif i.startswith("s_load"):
            if any(_sregs(t) & cur for t in toks[2:]):
                bad.add((k, str(i)))
            cur |= _sregs(toks[1])
        elif any(_sregs(t) & cur for t in toks[1:]):
            bad.add((k, str(i)))
        fs = frozenset(cur)
        for j in succ[k]:
            if state[j] is None or not fs <= state[j]:
                state[j] = fs if state[j] is None else state[j] | fs
                work.append(j)
    return sorted(bad)


def test_no_sgpr_use_while_scalar_load_in_flight(fast_kernels):
    bad = {k: inflight_scalar_load_hazards(v)[:3] for k, v in fast_kernels.items()}
    assert not any(bad.values()), {k: v for k, v in bad.items() if v}


def _vregs(tok):
    tok = tok.rstrip(",")
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


_LGKM = ("ds_", "s_load", "s_buffer_load", "s_sendmsg")


def inflight_lds_read_hazards(ins, cap=64):
    """Instructions that touch a VGPR while an LDS read writing it may still be in flight.

    The paired kernel's staged-entry reads can be hand-written ds_read_b64 (USV_PAIR_RDASM) that the
    compiler's waitcnt pass does not see, retired by explicit counted lgkmcnt waits; a register the
    compiler believes free (e.g. the never-read half of the last pair) would be clobbered by the late
    return.  Forward dataflow over the CFG with the ordered list of outstanding LDS operations (reads
    carry their destination VGPRs, other LDS operations none).  LDS operations return in order, so
    lgkmcnt(n) retires all but the n newest of them.  Scalar-memory loads and messages also count in
    lgkmcnt but return out of order (GFX9): one of them may have returned while n LDS operations are
    still pending, so they are NOT entries of the list -- counting one among "the n newest" would
    wrongly retire the LDS read just older than it.  A pending scalar load can only make a counted wait
    stricter for the LDS operations, never weaker, so leaving it out is the sound bound.
    """
    succ = _successors(ins)
    state = [None] * len(ins)
    state[0] = ()
    work, bad = [0], set()

    def join(a, b):
        n = max(len(a), len(b))
        a, b = ((frozenset(),) * (n - len(a)) + a, (frozenset(),) * (n - len(b)) + b)
        return tuple(x | y for x, y in zip(a, b))

    while work:
        k = work.pop()
        cur, i = list(state[k]), ins[k]
        toks = i.replace(",", " ").split()
        pend = set().union(*cur) if cur else set()
        if i.startswith("s_waitcnt") and "lgkmcnt" in i:
            n = int(re.search(r"lgkmcnt\((\d+)\)", i).group(1))
            cur = cur[len(cur) - n:] if n > 0 else []
        elif i.startswith(_LGKM):
            touched = set().union(*(_vregs(t) for t in toks[1:])) if len(toks) > 1 else set()
            if touched & pend:
                bad.add((k, str(i)))
            if i.startswith("ds_"):  # scalar loads / messages: out of order, not list entries (above)
                dst = _vregs(toks[1]) if i.startswith("ds_read") and len(toks) > 1 else set()
                cur.append(frozenset(dst))
                cur = cur[-cap:]
        elif i.startswith("v_"):
            if set().union(*(_vregs(t) for t in toks[1:])) & pend:
                bad.add((k, str(i)))
        fs = tuple(cur)
        for j in succ[k]:
            new = fs if state[j] is None else join(state[j], fs)
            if state[j] is None or new != state[j]:
                state[j] = new
                work.append(j)
    return sorted(bad)


def test_no_vgpr_use_while_lds_read_in_flight(fast_kernels):
    asm_reads = {k: v for k, v in fast_kernels.items() if "sad_pair_kernel" in k or "sad_group_kernel" in k or "ssd_fast_kernel" in k}
    bad = {k: inflight_lds_read_hazards(v)[:3] for k, v in asm_reads.items()}
    assert not any(bad.values()), {k: v for k, v in bad.items() if v}


def test_lds_read_hazard_checker_catches_a_clobber():
    # the round-4 defect this check exists for: the never-read half of a pending pair reused
    ins = [Insn(t, 4 * n) for n, t in enumerate([
        "ds_read_b64 v[10:11], v44", "ds_read_b64 v[28:29], v44 offset:72", "s_waitcnt lgkmcnt(1)",
        "v_sad_u8 v29, s40, v11, 0", "s_waitcnt lgkmcnt(0)", "s_endpgm"])]
    assert [k for k, _ in inflight_lds_read_hazards(ins)] == [3]
    ok = [Insn(t, 4 * n) for n, t in enumerate([
        "ds_read_b64 v[10:11], v44", "ds_write_b32 v1, v2", "s_waitcnt lgkmcnt(1)", "v_add_u32_e32 v3, v10, v11",
        "s_endpgm"])]
    assert inflight_lds_read_hazards(ok) == []


def test_lds_read_hazard_checker_scalar_loads_return_out_of_order():
    # lgkmcnt(1) with a scalar load as the newest LGKM operation: the s_load may have returned first,
    # leaving the second ds_read pending -- using its destination is a hazard (an in-order model that
    # counted the s_load as "the one still pending" would have passed this)
    bad = [Insn(t, 4 * n) for n, t in enumerate([
        "ds_read_b64 v[10:11], v44", "ds_read_b64 v[28:29], v44 offset:72", "s_load_dwordx2 s[4:5], s[0:1], 0x0",
        "s_waitcnt lgkmcnt(1)", "v_sad_u8 v30, s40, v28, 0", "s_waitcnt lgkmcnt(0)", "s_endpgm"])]
    assert [k for k, _ in inflight_lds_read_hazards(bad)] == [4]
    # an s_load between two reads: lgkmcnt(1) still retires the older read (LDS returns are in order)
    ok = [Insn(t, 4 * n) for n, t in enumerate([
        "ds_read_b64 v[10:11], v44", "s_load_dwordx2 s[4:5], s[0:1], 0x0", "ds_read_b64 v[28:29], v44 offset:72",
        "s_waitcnt lgkmcnt(1)", "v_sad_u8 v30, s40, v11, 0", "s_waitcnt lgkmcnt(0)", "s_endpgm"])]
    assert inflight_lds_read_hazards(ok) == []


def test_every_m0_write_feeds_an_lds_dma_or_addtid_store(fast_kernels):
    # The paired kernel's transpose stores (ds_write_addtid_b32) may address the LDS from the M0 value the row's
    # DMA left (USV_PAIR_M0REUSE): no instruction may write M0 unless it feeds, within two instructions, an
    # LDS-DMA or an addtid store (a compiler-inserted M0 write in between would redirect the stores).
    for name, ins in fast_kernels.items():
        for k, i in enumerate(ins):
            if re.match(r"s_\w+ m0,", i):
                nxt = ins[k + 1:k + 3]
                assert any(n.startswith(("global_load_lds", "ds_write_addtid")) or
                           (n.startswith("buffer_load") and n.endswith(" lds")) for n in nxt), (name, i, nxt)


def reaching_m0_writes(ins):
    """Forward dataflow over the CFG: for each instruction, the set of M0 writes (indices) that reach it."""
    succ = _successors(ins)
    state = [None] * len(ins)
    state[0] = frozenset()
    work = [0]
    while work:
        k = work.pop()
        out = frozenset({k}) if re.match(r"s_\w+ m0,", ins[k]) else state[k]
        for j in succ[k]:
            if state[j] is None or not out <= state[j]:
                state[j] = out if state[j] is None else state[j] | out
                work.append(j)
    return state


def test_addtid_stores_see_one_dma_m0(fast_kernels):
    # the static ring's transpose stores (USV_PAIR_M0REUSE) take M0 from the row's LDS-DMA.  Every
    # ds_write_addtid_b32 must be reached by exactly ONE M0 write on every CFG path, and that write must either
    # be an s_mov of the store group itself (the non-reuse form) or the M0 of an LDS-DMA (the row DMA whose base
    # the store's constant offset is computed against) -- never a join of different M0 values at a loop latch.
    n_reuse = 0
    for name, ins in fast_kernels.items():
        reach = reaching_m0_writes(ins)
        for k, i in enumerate(ins):
            if not i.startswith("ds_write_addtid"):
                continue
            r = reach[k]
            assert r is not None and len(r) == 1, (name, i, k, sorted(r or ()))
            (w,) = r
            nxt = ins[w + 1:w + 3]
            feeds_dma = any(n.startswith("global_load_lds") or (n.startswith("buffer_load") and n.endswith(" lds"))
                            for n in nxt)
            assert feeds_dma or ins[w].startswith("s_mov_b32 m0"), (name, i, ins[w])
            n_reuse += feeds_dma
    assert n_reuse > 0  # the reuse form is present in the build under test


def test_addtid_reuse_offsets_address_the_transpose_buffer(fast_kernels):
    # the reuse stores address tb as DMA M0 + offset, where the row DMA's M0 is
    # rbase + 4 NRS ((I + PD) mod NB) and the store offset D0 = 4 TB_OFF - 4 NRS ((I + PD) mod NB).  So for every
    # store group fed by a DMA's `s_add_u32 m0, <rbase>, <imm>` the sum imm + (first store's offset) is the same
    # constant (4 TB_OFF) in the whole kernel: a reordered or added DMA between a row's DMA and its stores, or a
    # slot / offset mismatch, breaks it.
    checked = 0
    for name, ins in fast_kernels.items():
        reach = reaching_m0_writes(ins)
        sums = set()
        for k, i in enumerate(ins):
            if not i.startswith("ds_write_addtid") or (k and ins[k - 1].startswith("ds_write_addtid")):
                continue
            (w,) = reach[k]
            m = re.match(r"s_add_u32 m0, s\d+, (0x[0-9a-f]+|\d+)$", ins[w])
            if not m:
                continue
            off = re.search(r"offset:(\d+)", i)
            sums.add(int(m.group(1), 0) + (int(off.group(1)) if off else 0))
            checked += 1
        assert len(sums) <= 1, (name, sorted(sums))
    assert checked > 0


def test_lds_dma_m0_wait_state(fast_kernels):
    # GFX9: an SALU write of M0 needs one wait state before an LDS-DMA reads it
    for name, ins in fast_kernels.items():
        for a, b in zip(ins, ins[1:]):
            if b.startswith("global_load_lds") or (b.startswith("buffer_load") and b.endswith(" lds")):
                assert not re.match(r"s_\w+ m0,", a), (name, a, b)


@pytest.fixture(scope="module")
def tiled_kernels(tmp_path_factory):
    funcs = _disassembly(tmp_path_factory.mktemp("isa_tiled"))
    tiled = {k: v for k, v in funcs.items() if "sad_tiled_kernel" in k}
    assert len(tiled) >= 2, sorted(tiled)  # SAD and SSD, every radius the dispatch instantiates
    return tiled


def test_tiled_no_scratch(tiled_kernels):
    bad = {k: sum("scratch_" in i for i in v) for k, v in tiled_kernels.items()}
    assert not any(bad.values()), {k: n for k, n in bad.items() if n}


def test_tiled_lds_dma_m0_wait_state(tiled_kernels):
    # the tiled kernel's ring (csrc/usv_sad_tiled.hip tdma) writes M0 in inline asm too
    n_dma = 0
    for name, ins in tiled_kernels.items():
        for a, b in zip(ins, ins[1:]):
            if b.startswith("global_load_lds") or (b.startswith("buffer_load") and b.endswith(" lds")):
                n_dma += 1
                assert not re.match(r"s_\w+ m0,", a), (name, a, b)
    assert n_dma > 0


def test_tiled_no_sgpr_use_while_scalar_load_in_flight(tiled_kernels):
    bad = {k: inflight_scalar_load_hazards(v)[:3] for k, v in tiled_kernels.items()}
    assert not any(bad.values()), {k: v for k, v in bad.items() if v}


def test_mfma_kernel_has_no_inline_asm_valu():
    # The compiler pads the MFMA wait states of its own instructions, not those of inline asm.  In round 5 a
    # variant of the SSD matrix kernel whose sel_mask() selects (inline-asm v_cndmask) were scheduled into an
    # MFMA's shadow wrote an operand register the MFMA was still reading and produced wrong maps; the product
    # kernel's selects are plain C++ since.  Keep every VALU of the MFMA kernel compiler-visible.
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "unsynchronized_stereo_vision_proj325_amd", "csrc", "usv_ssd_mfma.hip")).read()
    code = "\n".join(line.split("//")[0] for line in src.splitlines())
    assert "sel_mask(" not in code and "asm" not in code
