"""Register audit of the inline-asm MFMA chains in csrc/fused_seg4.hip (no GPU needed).

The input gradient's v_mfma_f32_16x16x32_bf16 groups are inline asm with VGPR accumulators
(fused_seg4.hip, the k-step loop): hipcc pads no hazard for them and sees their D registers as
written at the end of each statement.  The wait states the statements carry are safe only if
hipcc keeps the chain's accumulators where the asm left them -- the same four register ranges
in every group of a chain and no compiler instruction touching them between the first group
and the last (whose trailing s_nops cover the D -> VALU read).  The statements carry no pad for
a VALU write of an A / B operand (2 wait states): the check is that no VALU instruction among
the 2 before a statement writes one (they come from ds_reads, waited by hipcc's s_waitcnt).
Compiles the file to gfx950 assembly and checks exactly that, plus no scratch / spills."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "point-cloud-cnn-segmentation_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"), reason="no hipcc")


def vregs(text):
    """The arch VGPR numbers an instruction names (vN and v[a:b])."""
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for n in re.findall(r"(?<![\w\[])v(\d+)\b", text):
        out.add(int(n))
    return out


def compile_asm(tmp_path_factory, src, extra):
    """gfx950 assembly of csrc/<src> with csrc/Makefile's flags for it."""
    out = tmp_path_factory.mktemp("asm") / (src + ".s")
    cmd = [HIPCC if os.path.exists(HIPCC) else "hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "--cuda-device-only", "-S", *extra, "-o", str(out), src]
    subprocess.run(cmd, cwd=CSRC, check=True, capture_output=True)
    return out.read_text()


@pytest.fixture(scope="module")
def seg4_asm(tmp_path_factory):
    return compile_asm(tmp_path_factory, "fused_seg4.hip", ["-fno-slp-vectorize"])


# kernels whose LDS-DMA statements set M0 without restoring it (the file's comment at the DMA
# helper): hipcc's own code must never read or write M0 there
M0_FILES = {"fused_seg4.hip": ["-fno-slp-vectorize"], "gemm_glds.hip": ["-mllvm", "-disable-machine-sink"],
            "gram_glds.hip": ["-mllvm", "-disable-machine-sink"]}


@pytest.mark.parametrize("src", sorted(M0_FILES))
def test_compiler_code_leaves_m0_alone(tmp_path_factory, src):
    asm = compile_asm(tmp_path_factory, src, M0_FILES[src])
    inasm, uses = False, []
    for ln in asm.splitlines():
        t = ln.strip()
        if t == ";;#ASMSTART":
            inasm = True
        elif t == ";;#ASMEND":
            inasm = False
        elif not inasm and not t.startswith(";") and re.search(r"\bm0\b", t.split(";")[0]):
            uses.append(t)
    assert not uses, uses[:5]


def kernels(asm):
    for m in re.finditer(r"^(_ZN\w*seg4_kernel\w*):", asm, flags=re.M):
        end = asm.index(".Lfunc_end", m.end())
        yield m.group(1), asm[m.end():end]


def chains(body):
    """Yield (groups, between): each group the list of D ranges of one asm MFMA statement, and
    the compiler lines between the chain's first and last statements."""
    lines = [ln.strip() for ln in body.splitlines()]
    i, groups, between, in_chain = 0, [], [], False
    while i < len(lines):
        if lines[i] == ";;#ASMSTART":
            j = lines.index(";;#ASMEND", i)
            stmt = lines[i + 1:j]
            mf = [s for s in stmt if s.startswith("v_mfma_f32_16x16x32_bf16")]
            if mf:
                ds = [s.split()[1].rstrip(",") for s in mf]
                starts = all(s.rstrip().endswith(", 0") for s in mf)
                if starts:
                    assert not in_chain, "a chain restarted before its closing group"
                    in_chain, groups, between = True, [], []
                assert in_chain, "an accumulate group outside a chain"
                groups.append(ds)
                if any(s.startswith("s_nop 7") for s in stmt):
                    yield groups, between
                    in_chain = False
            elif in_chain:
                between.extend(stmt)
            i = j + 1
            continue
        if in_chain and lines[i] and not lines[i].startswith(";") and not lines[i].startswith("."):
            between.append(lines[i])
        i += 1
    assert not in_chain, "a chain without its closing group"


def test_seg4_asm_chains_keep_their_accumulators(seg4_asm):
    seen = 0
    for name, body in kernels(seg4_asm):
        n = 0
        for groups, between in chains(body):
            n += 1
            assert all(g == groups[0] for g in groups), (name, groups)
            d = set()
            for r in groups[0]:
                d |= vregs(r)
            assert len(d) == 16, (name, groups[0])
            touch = [ln for ln in between if vregs(ln) & d]
            assert not touch, (name, touch[:5])
        assert n >= 1, name
        seen += 1
    assert seen == 4   # <128, 256> and <256, 512>, dropout mask on / off


def operand_hazards(body):
    """(statement, instruction) pairs where one of the 2 instructions before an asm MFMA
    statement is a VALU write of one of its A / B operands."""
    lines = [ln.strip() for ln in body.splitlines()]
    bad = []
    for i, ln in enumerate(lines):
        if ln != ";;#ASMSTART":
            continue
        j = lines.index(";;#ASMEND", i)
        mf = [s for s in lines[i + 1:j] if s.startswith("v_mfma_f32_16x16x32_bf16")]
        if not mf:
            continue
        ins = set()
        for s in mf:
            ops = [o.strip() for o in s.split(None, 1)[1].split(",")]
            ins |= vregs(ops[1]) | vregs(ops[2])
        seen, k = 0, i - 1
        while seen < 2 and k >= 0:
            prev = lines[k]
            k -= 1
            if not prev or prev.startswith(";") or prev.startswith("."):
                continue
            if prev.endswith(":"):
                bad.append((mf[0], "a label: control may arrive without the wait states"))
                break
            seen += 1
            if prev.startswith("v_") and not prev.startswith("v_mfma"):
                dst = prev.split(None, 1)[1].split(",")[0] if " " in prev else ""
                if vregs(dst) & ins:
                    bad.append((mf[0], prev))
    return bad


def test_seg4_asm_operands_not_fresh_from_valu(seg4_asm):
    for name, body in kernels(seg4_asm):
        bad = operand_hazards(body)
        assert not bad, (name, bad[:3])


def test_seg4_no_scratch(seg4_asm):
    spills = re.findall(r"\.vgpr_spill_count:\s+(\d+)", seg4_asm)
    scratch = re.findall(r"\.private_segment_fixed_size:\s+(\d+)", seg4_asm)
    assert spills and scratch
    assert all(int(v) == 0 for v in spills + scratch)


def test_audit_catches_the_patterns_it_guards():
    """The parsers above flag what they are meant to flag (synthetic assembly, no compiler)."""
    moved = """
;;#ASMSTART
v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], 0
;;#ASMEND
v_mov_b32_e32 v20, v2
;;#ASMSTART
v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], v[0:3]
s_nop 7
s_nop 3
;;#ASMEND
"""
    (groups, between), = list(chains(moved))
    assert [ln for ln in between if vregs(ln) & vregs(groups[0][0])] == ["v_mov_b32_e32 v20, v2"]
    fresh = """
v_add_u32_e32 v9, v1, v2
;;#ASMSTART
v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], 0
;;#ASMEND
"""
    assert operand_hazards(fresh) == [("v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], 0",
                                       "v_add_u32_e32 v9, v1, v2")]
    padded = """
v_add_u32_e32 v9, v1, v2
s_waitcnt lgkmcnt(0)
s_mov_b32 s1, s2
;;#ASMSTART
v_mfma_f32_16x16x32_bf16 v[0:3], v[8:11], v[12:15], 0
;;#ASMEND
"""
    assert operand_hazards(padded) == []
    assert vregs("v_pk_fma_f32 v[70:71], v[198:199], v3, v[190:191]") == {70, 71, 198, 199, 3, 190, 191}
