"""ISA invariant of the direct-B tile GEMM (csrc/bwd_gemm.hip, tile_gemm_db_kernel), checked on
the compiler's own output (hipcc -S for gfx950; no GPU needed).

The kernel's B fragments are loaded by inline-asm global_load_dwordx4 that hipcc does not count
for its waitcnt insertion; the counted s_waitcnt before each stage's barrier retires them. That is
only sound if nothing reads or writes a ring register between its load and that wait -- in
particular no compiler-inserted copy (v_mov / v_accvgpr / v_perm ...) of an in-flight register,
which hipcc would place right after the definition. The test checks that straight-line window
after every ring load (see the test's docstring for what it does not model)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "triad_amd", "csrc")


def _regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def _kernels(asm):
    """{symbol: [instruction lines]} of the tile_gemm_db kernels."""
    out, cur = {}, None
    for line in asm.splitlines():
        if re.match(r"^_Z\S*tile_gemm_db(16)?_kernel\S*:", line):
            cur = line.split(":")[0]
            out[cur] = []
        elif cur is not None:
            if line.strip().startswith("s_endpgm"):
                cur = None
            else:
                out[cur].append(line)
    return out


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "bwd_gemm.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-I", CSRC, "-I", os.path.join(ROOT, "include"), "-Xclang", "-target-feature", "-Xclang",
                    "-packed-fp32-ops", os.path.join(CSRC, "bwd_gemm.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


def _parse(lines):
    """[(kind, op, operands)] with kind "ringload" for the inline-asm B loads and "label" for
    branch targets."""
    out, asm_block = [], False
    for raw in lines:
        t = raw.strip()
        if re.match(r"^\.LBB\S*:", t):
            out.append(("label", t.split(":")[0], []))
            continue
        if t.startswith(";;#ASMSTART"):
            asm_block = True
            continue
        if t.startswith(";;#ASMEND"):
            asm_block = False
            continue
        s = t.split(";")[0].strip()
        if not s or s.endswith(":") or s.startswith("."):
            continue
        parts = s.replace(",", " ").split()
        op, ops = parts[0], parts[1:]
        out.append(("ringload" if asm_block and op == "global_load_dwordx4" else "other", op, ops))
    return out


def _touches(op, ops, regs):
    """Does the instruction read or write any of regs? (every register operand counts)"""
    return bool(set().union(set(), *(_regs(t) for t in ops)) & regs)


def test_direct_b_ring_registers_untouched_after_their_load(asm):
    """After each ring load into registers R, up to the next branch or barrier (the straight-line
    code where hipcc would place a copy of a freshly defined value): no instruction but another
    ring load into other registers may read or write R. The consuming MFMAs come after the stage's
    counted wait and barrier; beyond the first branch the walk would need the loop's control flow
    (the exit path reuses these registers once no load is in flight), which this check does not
    model -- the bit-identity GPU test (test_tile_gemm_packed_bit_identical_to_ring) covers it."""
    kernels = _kernels(asm)
    assert len(kernels) == 8, list(kernels)   # dQ / dK x direct / slab output, 32x32x16 and 16x16x32
    windows = 0
    for name, lines in kernels.items():
        inst = _parse(lines)
        for i, (kind, op, ops) in enumerate(inst):
            if kind != "ringload":
                continue
            regs = _regs(ops[0])
            windows += 1
            for kind2, op2, ops2 in inst[i + 1:]:
                if kind2 == "label" or op2.startswith("s_cbranch") or op2.startswith("s_branch") or \
                        op2 in ("s_barrier", "s_endpgm"):
                    break
                if kind2 == "ringload" and not (_regs(ops2[0]) & regs):
                    continue
                assert not _touches(op2, ops2, regs), (name, op, ops, "then", op2, ops2)
    assert windows >= 8 * 8, windows
