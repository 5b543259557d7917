"""Build a probe variant of the whole library: a copy of csrc/ with text replacements applied, compiled into
tools/probe/build/lib_<name>.so (load it with ARCWELD_LIB=...).  The product source carries no probe switches; the
variants live here.  Results of a variant are not the product's (it leaves work out).
usage (CPU side): python tools/probe/lib_variant.py <name>"""
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")

# name -> [(file, product text, replacement)]
VARIANTS = {
    "base": [],
    # the fused un-patch head forward + pass 1 without its per-channel sums' global atomics (7H per workgroup)
    "head_noatom": [("vqvae.hip", "    if (i < 5 * H) {\n      atomicAdd(gw2 + i, t);",
                     "    if (t == -1.2345f) {\n      atomicAdd(gw2 + i, t);")],
}


def main():
    name = sys.argv[1]
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
