"""Build a probe variant of the whole library: a copy of csrc/ with text replacements applied, compiled into
tools/probe/build/lib_<name>.so (load it with ARCWELD_LIB=...).  The product source carries no probe switches; the
variants live here.  Results of a variant are not the product's (it leaves work out).
usage (CPU side): python tools/probe/lib_variant.py <name>"""
import glob
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")

# name -> [(file, product text, replacement)]
VARIANTS = {
    "base": [],
    # the decoder chain's images with the encoder's swizzle keys (key(u) = u: the round-5 layout before the search)
    "chain_oldkeys": [("reschain.hip", "0xfdb64fdb98264210ull", "0xfedcba9876543210ull")],
    # the fused un-patch head forward + pass 1 without its per-channel sums' global atomics (7H per workgroup)
    "head_noatom": [("vqvae.hip", "  for (int i0 = threadIdx.x; i0 < 7 * H; i0 += 64 * HFW) {",
                     "  for (int i0 = threadIdx.x; i0 < 7 * H && gmul < -1e30f; i0 += 64 * HFW) {")],
}


# a bounds guard: an index compared with a limit (`i0 < 7 * H`, `row < nrows`), up to the clause's end
GUARD = re.compile(r"\b[A-Za-z_]\w*(?:\[[^\]]*\])?\s*(?:<=|>=|<|>)\s*[\w\s*+\-()]+?(?=\s*(?:;|&&|\|\||\)\s*[{;]|$))")


def kept_guards(a, b):
    """The guards of the product text `a` that its replacement `b` drops (a variant may add conditions to a guard,
    never remove or rewrite one: round 5's first head_noatom replaced `i < 5 * H` and indexed below its array)."""
    return [g.strip() for g in GUARD.findall(a) if g.strip() not in b]


def check(name):
    for fn, a, b in VARIANTS[name]:
        lost = kept_guards(a, b)
        if lost:
            sys.exit(f"{name}: the replacement in {fn} drops bounds guard(s) {lost}")


def main():
    name = sys.argv[1]
    check(name)
    work = os.path.join(HERE, "build", "src_" + name)
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    for f in glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) + [
            os.path.join(CSRC, "Makefile")]:
        shutil.copy(f, work)
    inc = os.path.join(REPO, "include", "arcweld_amd.h")
    for fn in ("common.h", "Makefile"):   # the copy's relative paths to include/
        p = os.path.join(work, fn)
        s = open(p).read().replace("../../include/arcweld_amd.h", inc).replace("-I../../include",
                                                                               "-I" + os.path.dirname(inc))
        open(p, "w").write(s)
    for fn, a, b in VARIANTS[name]:
        p = os.path.join(work, fn)
        s = open(p).read()
        if s.count(a) != 1:
            sys.exit(f"{name}: text not found exactly once in {fn}: {a[:60]!r}")
        open(p, "w").write(s.replace(a, b))
    out = os.path.join(HERE, "build", f"lib_{name}.so")
    subprocess.check_call(["make", "-s", "-j8", f"OUT={out}", f"OBJDIR={work}/obj"], cwd=work)
    shutil.rmtree(work, ignore_errors=True)
    print("built", out)


if __name__ == "__main__":
    main()
