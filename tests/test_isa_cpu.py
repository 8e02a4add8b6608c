"""ISA invariants of the library's hand-scheduled kernels, checked on the compiler's own output
(hipcc -S for gfx950 with the product flags; no GPU needed).

1. No register load hidden from hipcc. An inline-asm load with a VGPR destination is absent from
   hipcc's waitcnt bookkeeping and its destination counts as written at ;;#ASMEND, so the
   compiler may copy, spill or reuse the register before the data lands
   (cdna_hip_programming.md §5.7 item 1). Round 4's direct-B tile GEMM did exactly that in a build
   with more register pressure (the TRIAD_LDS_CHECK printf build spilled each ring register right
   after its load and reused it: HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION,
   gpurun_out/r04d_py5.log). Every asm statement of the library may only load into LDS
   (global_load_lds_*, buffer_load_* ... lds) or wait / barrier / move M0; register loads are
   ordinary loads hipcc counts.
2. No scratch in any kernel that issues LDS-DMA: `.private_segment_fixed_size 0` and
   `.vgpr_spill_count 0` (a spilled kernel is not wrong by itself once no load is hidden, but
   these kernels' schedules assume their register budget; a spill is a silent performance
   cliff and the first sign that a budget assumption broke).
3. The direct-B tile GEMM keeps its B prefetch in flight: in the steady-state loop every wait hipcc
   emits before an MFMA leaves >= 8 loads outstanding (two stages of four B loads), i.e. the
   restructured loop (whole groups of stages, no exit inside, unconditional prefetch) lets hipcc
   count exactly instead of draining the ring at a merge point.
4. Every hand-counted wait matches what hipcc emitted: the forward's sync_tile constants are
   re-derived from the LDS-DMA pieces and dS stores per tile found in its stage loop, and every
   tail stage of the direct-B and row-panel GEMMs drains (vmcnt(0)) before its barrier. Each check
   fails when a counted constant is edited by one (verified by hand)."""
import concurrent.futures as cf
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "triad_amd", "csrc")


def _sources_with_asm():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip"):
            text = open(os.path.join(CSRC, f)).read()
            if "asm" in text or "glds16" in text or "global_load_lds" in text:
                out.append(f)
    return out


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    """{source file: hipcc -S output} for every source with inline asm or LDS-DMA."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    import sys
    sys.path.insert(0, ROOT)
    from triad_amd import build
    d = tmp_path_factory.mktemp("isa")
    flags = [f for f in build.FLAGS if f != "-fPIC"]

    def one(f):
        out = d / (f + ".s")
        subprocess.run([hipcc, *flags, *build.EXTRA.get(f, []), "--cuda-device-only", "-S",
                        os.path.join(CSRC, f), "-o", str(out)], check=True, capture_output=True)
        return f, out.read_text()

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        return dict(ex.map(one, _sources_with_asm()))


def _kernels(asm):
    """{symbol: [instruction lines]} of every kernel in one .s file."""
    names = set(re.findall(r"^\s+\.amdhsa_kernel (\S+)", asm, re.M))
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^(\S+):", line)
        if m and m.group(1) in names:
            cur = m.group(1)
            out[cur] = []
        elif cur is not None:
            if line.strip().startswith(".Lfunc_end"):   # a kernel may have several s_endpgm exits
                cur = None
            else:
                out[cur].append(line.strip())
    return out


def _meta(asm, sym):
    m = re.search(r"\.name:\s+" + re.escape(sym) + r"\n((?:\s+\..*\n)+)", asm)
    block = m.group(1) if m else ""
    get = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", block).group(1))  # noqa: E731
    return get("private_segment_fixed_size"), get("vgpr_spill_count")


_REG_LOAD = re.compile(r"^(global_load_|buffer_load_|flat_load_|scratch_load_|ds_read|ds_load)")


def test_no_register_load_hidden_in_inline_asm(isa):
    """Every load inside an inline-asm statement writes LDS, not VGPRs."""
    asm_stmts = 0
    for f, asm in isa.items():
        inside = False
        for line in asm.splitlines():
            t = line.strip()
            if t.startswith(";;#ASMSTART"):
                inside, asm_stmts = True, asm_stmts + 1
                continue
            if t.startswith(";;#ASMEND"):
                inside = False
                continue
            if not inside:
                continue
            op = t.split(";")[0].strip()
            if _REG_LOAD.match(op):
                lds_dma = op.startswith("global_load_lds_") or re.search(r"\blds\b", op)
                assert lds_dma, (f, op)
    assert asm_stmts > 100, asm_stmts


def test_lds_dma_kernels_have_no_scratch(isa):
    """Zero private segment and zero VGPR spills for every kernel that issues LDS-DMA."""
    checked = []
    for f, asm in isa.items():
        for sym, lines in _kernels(asm).items():
            if not any(l.startswith("global_load_lds_") or (l.startswith("buffer_load_") and " lds" in l)
                       for l in lines):
                continue
            priv, spills = _meta(asm, sym)
            assert (priv, spills) == (0, 0), (f, sym, priv, spills)
            checked.append(sym)
    assert len(checked) >= 30, len(checked)


def test_direct_b_loop_keeps_b_prefetch_in_flight(isa):
    """tile_gemm_db16_kernel: inside the stage loop (its loop header to the back branch) every
    compiler wait leaves >= 8 vector-memory ops outstanding except the explicit counted waits
    (inline asm, retiring the A LDS-DMA before each barrier), and every stage issues its four B
    loads as ordinary instructions."""
    asm = isa["bwd_gemm.hip"]
    ks = {s: l for s, l in _kernels(asm).items() if "tile_gemm_db16_kernel" in s}
    assert len(ks) == 4, list(ks)   # dQ / dK x direct / slab output
    for sym, lines in ks.items():
        hdr = next(i for i, l in enumerate(lines) if "Loop Header" in l)
        label = lines[hdr].split(":")[0]
        back = max(i for i, l in enumerate(lines) if re.match(r"s_(cbranch_\w+|branch)\s+" + re.escape(label) + r"$", l))
        body, inside, waits, bloads, stages = lines[hdr:back], False, [], 0, 0
        for l in body:
            if l.startswith(";;#ASMSTART"):
                inside = True
            elif l.startswith(";;#ASMEND"):
                inside = False
            elif l.startswith("s_barrier"):
                stages += 1
            elif l.startswith("global_load_dwordx4") and not inside:
                bloads += 1
            else:
                m = re.match(r"s_waitcnt\s.*vmcnt\((\d+)\)", l)
                if m and not inside:
                    waits.append(int(m.group(1)))
        assert stages == 4, (sym, stages)          # one group of NB = 4 stages per iteration
        assert bloads == 4 * stages, (sym, bloads)
        assert waits and min(waits) >= 8, (sym, waits)
        priv, spills = _meta(asm, sym)
        assert (priv, spills) == (0, 0), (sym, priv, spills)


def test_direct_b_tail_stages_drain_before_their_barrier(isa):
    """Direct-B tile GEMMs (tile_gemm_db16_kernel): after the stage loop's back
    branch, the trailing nst % NB stages issue no B loads (their prefetch feeds no later stage, so
    hipcc removes it), so the loop's counted wait would under-count the VMEM ops in flight (round 5:
    AV dK with a 2-stage tail was non-deterministic). Every barrier there must follow a vmcnt(0)."""
    checked = 0
    # (the row-panel kernels' tails: test_rowgemm_tail_stages_drain_before_their_barrier)
    for f, pat in (("bwd_gemm.hip", "tile_gemm_db16_kernel"),):
        for sym, lines in _kernels(isa[f]).items():
            if pat not in sym or not any("Loop Header" in l for l in lines):
                continue
            hdr = next(i for i, l in enumerate(lines) if "Loop Header" in l)
            label = lines[hdr].split(":")[0]
            back = max(i for i, l in enumerate(lines)
                       if re.match(r"s_(cbranch_\w+|branch)\s+" + re.escape(label) + r"$", l))
            last_vm = None
            tail_barriers = 0
            for l in lines[back + 1:]:
                m = re.match(r"s_waitcnt\s.*vmcnt\((\d+)\)", l)
                if m:
                    last_vm = int(m.group(1))
                elif l.startswith("s_barrier"):
                    tail_barriers += 1
                    assert last_vm == 0, (f, sym, last_vm)
            assert tail_barriers >= 1, (f, sym)
            checked += 1
    assert checked >= 4, checked


def _loop_span(lines):
    """(header index, back-branch index) of the kernel's first loop."""
    hdr = next(i for i, l in enumerate(lines) if "Loop Header" in l)
    label = lines[hdr].split(":")[0]
    back = max(i for i, l in enumerate(lines) if re.match(r"s_(cbranch_\w+|branch)\s+" + re.escape(label) + r"$", l))
    return hdr, back


def _loop_lines(lines, hdr=None):
    """Indices of the lines of one loop (default: the kernel's first): the header block and every
    block hipcc annotates as in that loop (some are placed after the back branch)."""
    if hdr is None:
        hdr = next(i for i, l in enumerate(lines) if "Loop Header" in l)
    tag = "Header=" + lines[hdr].split(":")[0].lstrip(".L")
    out, inside = [], False
    for i, l in enumerate(lines):
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", l):
            inside = i == hdr or (tag in l and "in Loop" in l)
        if inside:
            out.append(i)
    return out


def _asm_runs(lines, lo, hi, idx=None):
    """Inside lines[lo:hi] (or at the indices idx): the runs of inline-asm VMEM ops ('D' = LDS-DMA piece, 'S' = store),
    each run a maximal sequence of one kind with no other VMEM op or label between, as
    (kind, count, first line); and the immediates of the inline-asm `s_waitcnt vmcnt(N)`."""
    runs, waits, inside = [], [], False
    for i in (range(lo, hi) if idx is None else idx):
        t = lines[i]
        if t.startswith(";;#ASMSTART"):
            inside = True
            continue
        if t.startswith(";;#ASMEND"):
            inside = False
            continue
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:|s_branch |s_cbranch_)", t):   # a block boundary ends a run
            runs.append(("|", 0, i))
            continue
        if not t or t[0] in ";.":
            continue
        op = t.split()[0]
        m = re.match(r"s_waitcnt\s.*vmcnt\((\d+)\)", t)
        if m and inside:
            waits.append(int(m.group(1)))
        if not re.match(r"(global_|buffer_|flat_|scratch_)(load|store|atomic)", op):
            continue
        if inside and (op.startswith("global_load_lds") or (op.startswith("buffer_load") and re.search(r"\blds\b", t))):
            k = "D"
        elif inside and "_store" in op:
            k = "S"
        else:
            k = "x"   # an ordinary (compiler-counted) VMEM op
        if runs and runs[-1][0] == k:
            runs[-1] = (k, runs[-1][1] + 1, runs[-1][2])
        else:
            runs.append((k, 1, i))
    return [r for r in runs if r[0] != "|"], waits


def test_forward_counted_waits_match_emitted_vmem(isa):
    """The training forward's sync_tile (pairsim_fwd.hip) hand-counts its vmcnt: younger than the
    key tile about to be read are the DMA pieces of nd = min(1, tiles left) later tiles and the dS
    stores of ns = min(1, b - 1) earlier epilogues, so it waits vmcnt(nd G + ns S) for G pieces per
    tile and S stores per epilogue. Here G and S are read off what hipcc emitted: every prefetch in
    the stage loop is one run of G asm LDS-DMA pieces, every epilogue one run of S asm stores, the
    runs alternate (a tile's pieces before the next epilogue's stores, nothing counted between), and
    the counted waits in the loop are exactly {nd G + ns S} -- a constant off by one, a piece or a
    store hipcc dropped or duplicated, or a reordering fails. The prologue's sync_tile(0) waits
    vmcnt(nd G) after exactly NBUF - 1 = 2 prefetches. The loop runs two tiles per trip (the
    accumulator sets alternate, TRIAD_FWD_PINGPONG); an odd last tile runs in straight-line code
    after it, whose counted waits must decode to some (nd, ns) as well."""
    asm = isa["pairsim_fwd.hip"]
    ks = {s: l for s, l in _kernels(asm).items()
          if ("pairsim_fwd2_kernelILb1E" in s or "pairsim_fwd_multi_kernelILb1E" in s)}
    assert len(ks) == 3, list(ks)   # training: fwd2 <SHORTQ 0/1>, multi
    for sym, lines in ks.items():
        # one stage loop per training body (the fast and the exact epilogue, FwdArgs::exact)
        hdrs = [i for i, l in enumerate(lines) if "Loop Header" in l and "Depth=1" in l]
        assert len(hdrs) == 2, (sym, len(hdrs))
        prev = 0
        allruns, allwaits = _asm_runs(lines, 0, len(lines))
        for hdr in hdrs:
            loop = _loop_lines(lines, hdr)
            runs, waits = _asm_runs(lines, 0, 0, loop)
            d_runs = [n for k, n, _ in runs if k == "D"]
            s_runs = [n for k, n, _ in runs if k == "S"]
            assert d_runs and s_runs and len(set(d_runs)) == 1 and len(set(s_runs)) == 1, (sym, runs)
            G, S = d_runs[0], s_runs[0]
            assert (G, S) == (4, 2), (sym, G, S)   # GLDS_PER_TILE = 32 / WAVES; two 1 KB stores per tile
            kinds = [k for k, _, _ in runs if k in "DS"]
            assert kinds == ["D", "S"] * (len(kinds) // 2), (sym, kinds)
            assert set(waits) == {0, G, S, G + S}, (sym, sorted(set(waits)), (G, S))
            # this body's prologue: the code outside any loop since the previous body's last dS
            # store (hipcc may hoist the prologue prefetches both bodies share above the branch
            # between them: then only the first body's region holds them)
            inloop = set(loop)
            pro = [i for i in range(prev, hdr) if i not in inloop]
            pro_runs, _ = _asm_runs(lines, 0, 0, pro)
            last_s = max([ln for k, _, ln in pro_runs if k == "S"], default=-1)
            pro = [i for i in pro if i > last_s]
            pro_runs, pro_waits = _asm_runs(lines, 0, 0, pro)
            pro_d = [n for k, n, _ in pro_runs if k == "D"]
            assert pro_d and set(pro_d) == {G} and set(pro_waits) <= {0, G}, (sym, pro_runs, pro_waits)
            if prev == 0:
                assert pro_d[:2] == [G, G], (sym, pro_runs)
            prev = max(loop) + 1
        # everywhere (the odd-tile step after each loop included): pieces come G per tile, stores S
        # per epilogue, and every counted wait is one of nd G + ns S
        assert {n for k, n, _ in allruns if k == "D"} == {G} and {n for k, n, _ in allruns if k == "S"} == {S}, sym
        assert set(allwaits) <= {0, G, S, G + S}, (sym, sorted(set(allwaits)))


def test_rowgemm_tail_stages_drain_before_their_barrier(isa):
    """The row-panel projection GEMMs (rowgemm.hip) run whole groups of stages in the loop and the
    trailing ones in straight-line code, like the direct-B tile GEMM; their B prefetches feed no
    later stage there, so hipcc removes them and a counted wait would under-count (round 5's race).
    Every barrier after the loop that is followed by MFMA work (a tail stage, or the fused form's
    second GEMM from the LDS panel) must follow a vmcnt(0); the epilogue's own barriers (LDS
    reductions, no MFMA) are not stages."""
    checked = 0
    for sym, lines in _kernels(isa["rowgemm.hip"]).items():
        if not any("Loop Header" in l for l in lines):
            continue
        _, back = _loop_span(lines)
        tail = lines[back + 1:]
        last_vm, stages = None, 0
        for i, l in enumerate(tail):
            m = re.match(r"s_waitcnt\s.*vmcnt\((\d+)\)", l)
            if m:
                last_vm = int(m.group(1))
            elif l.startswith("s_barrier"):
                nxt = next((j for j in range(i + 1, len(tail)) if tail[j].startswith("s_barrier")), len(tail))
                if any(t.startswith("v_mfma") for t in tail[i + 1:nxt]):
                    stages += 1
                    assert last_vm == 0, (sym, i, last_vm)
        assert stages >= 1, sym
        checked += 1
    assert checked >= 4, checked
