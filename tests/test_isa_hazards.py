"""ISA audit of the shipped kernels (CPU: hipcc cross-compiles gfx950 device assembly here): no VALU instruction
overwrites the data registers of a wide (> 64-bit) vector-memory store with fewer than 2 wait states behind it.

gfx94x / gfx950 need 2 wait states there (LLVM GCNHazardRecognizer: VALUWaitStates = 2; cdna_hip_programming.md 5.7
item 1).  ROCm 7.2's hazard recognizer pads every form except a MUBUF / MTBUF store whose soffset is a register, and
the fused ResBlock chains (csrc/reschain.hip ec_store16) store with an SGPR soffset: unpadded, the compiler put the
next LDS address into the first data register on the very next instruction, and the stored line's first dword
intermittently came out as that address on the GPU (round 5).  The chain pads each such store itself; this test
keeps the whole library honest after every edit, whatever the compiler's register allocation does."""
import os
import re
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

WIDE_STORE = re.compile(r"(buffer|global|flat)_store_(dwordx3|dwordx4|b96|b128)\b")


def _regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _wait_states(ins):
    m = re.match(r"s_nop\s+(\d+)", ins)
    return int(m.group(1)) + 1 if m else 1


def hazards(asm_lines):
    """(store, writer, wait states) for every VALU write of a wide store's data VGPRs within 2 wait states of the
    store, along the fall-through path (a label or s_endpgm ends the scan: the next block is not a successor)."""
    lines = [ln.split(";")[0].strip() for ln in asm_lines]
    out = []
    for i, ln in enumerate(lines):
        op = ln.split()[0] if ln else ""
        if not WIDE_STORE.match(op):
            continue
        ops = [t.strip() for t in ln.split(None, 1)[1].split(",")]
        data = _regs(ops[1] if op.startswith(("global", "flat")) else ops[0])
        w = 0
        for s in lines[i + 1:i + 12]:
            if not s or s.startswith("."):
                continue
            if s.endswith(":") or s.startswith("s_endpgm") or s.startswith("s_branch"):
                break
            o = s.split()[0]
            if o.startswith("v_") and data & _regs(s.split(None, 1)[1].split(",")[0].strip()):
                out.append((ln, s, w))
                break
            w += _wait_states(s)
            if w >= 2:
                break
    return out


def test_scanner_flags_the_round5_pattern():
    bad = ["buffer_store_dwordx4 v[34:37], v217, s[24:27], s65 offen sc1", "v_add_u32_e32 v34, 0xc008, v222"]
    assert len(hazards(bad)) == 1
    padded = [bad[0], "s_nop 1", bad[1]]
    assert hazards(padded) == []
    narrow = ["buffer_store_dwordx2 v[34:35], v217, s[24:27], s65 offen", "v_add_u32_e32 v34, 0xc008, v222"]
    assert hazards(narrow) == []
    other_block = [bad[0], "s_endpgm", ".LBB2_31:", bad[1]]
    assert hazards(other_block) == []


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_library_has_no_unpadded_wide_store_data_hazard():
    # the sources whose wide stores the compiler cannot pad on its own: MUBUF store builtins (an SGPR soffset is
    # possible) and inline-asm stores (hipcc pads nothing inside an asm string); every other store is compiler-emitted
    # global_store with soffset-free addressing, which the hazard recognizer pads (the whole library was scanned
    # clean once, round 6: 5 min of compiles, too long for every CPU run)
    pat = re.compile(r"raw_buffer_store|_store_dwordx[34]|aw_st_wt\(")
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip") and pat.search(open(os.path.join(CSRC, f)).read()))
    assert "reschain.hip" in srcs
    with tempfile.TemporaryDirectory() as tmp:
        def build(f):
            out = os.path.join(tmp, f + ".s")
            subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                            "-I" + os.path.join(REPO, "include"), "-S", "--cuda-device-only",
                            os.path.join(CSRC, f), "-o", out], check=True, capture_output=True, cwd=CSRC)
            with open(out) as fh:
                return f, hazards(fh.readlines())
        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            found = {f: h for f, h in ex.map(build, srcs) if h}
    assert not found, f"wide-store data overwritten within 2 wait states: {found}"
