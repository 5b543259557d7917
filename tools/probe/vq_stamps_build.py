"""Build tools/probe/build/vqs.so: a probe copy of csrc/vq.hip whose codebook-pinned forward writes s_memtime stamps
at its phase boundaries (thread 0 of the first 256 workgroups, vector stores into a __device__ buffer), plus
`vq_probe_stamps(uint64_t out[256 * 8])`.  The product source carries no probe code; the stamps are spliced in here
at fixed anchors (the build fails if one is missing).  Read by tools/probe/vq_stamps_probe.py on the GPU box.
usage (CPU side): python tools/probe/vq_stamps_build.py [variant]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "vq-vae-transformer-arc-welding_amd", "csrc")
OUT = os.path.join(HERE, "build")

# lane 0 of every wave stamps ([256 workgroups][8 waves][16 slots]); the scheduling barriers keep the compiler from
# moving work across a stamp
STAMP = ("__builtin_amdgcn_sched_barrier(0); if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) "
         "vq_stamp_buf[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + {n}] = __builtin_amdgcn_s_memtime(); "
         "__builtin_amdgcn_sched_barrier(0);")
RTIME = ("if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) "
         "vq_stamp_buf[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + {n}] = __builtin_amdgcn_s_memrealtime();")

# (anchor text inside vq_fwd_pinned_kernel, stamp index, where): "after" = after the anchor's first line,
# "before" = before the anchor, "end" = before the kernel's closing brace (the anchor is the kernel's last lines).
# Slots 0-6 are shader-clock phase stamps, 8 / 9 the 100 MHz real-time clock at start / end.
ANCHORS = [
    ("  const int64_t row0 = (int64_t)blockIdx.x * ROWS;\n\n  // ---- loads", [0, 8], "after"),
    ("  // ---- chunk loop", [1], "before"),
    ("  ees[tid] = tid < K ? ee", [2], "before"),
    ("  // ---- distances d = fl(", [3], "before"),
    ("  // ---- lexicographic (d, k) merge", [4], "before"),
    ("  // ---- thread (row r, quad q) reads its row's winner", [5], "before"),
    ("    atomicAdd(sqerr, t);\n  }\n}", [6, 9], "end"),
]
PHASES = "loads-issue+z chunks(mfma) norms-publish argmin merge+barrier finish"

# probe variants (results of a variant are not the product's): name -> [(product text, replacement)]
VARIANTS = {
    "base": [],
    # no same-address f64 atomic at the end of every workgroup
    "nosq": [("  if (tid == 0) {\n    double t = 0.0;", "  if (tid == 0 && red[1] == -1.0) {\n    double t = 0.0;")],
    # z_q stored write-through (sc1): its lines leave L2 during the kernel, not at the end-of-kernel release
    "wt": [("    reinterpret_cast<float4*>(zq + row * D)[q] = o;\n    if (zq2) {",
            "    aw_st_wt(zq + row * D + 4 * q, f32x4{o.x, o.y, o.z, o.w});\n    if (zq2) {")],
    # launch floor: the workgroups exit at once (same LDS allocation and grid)
    "empty": [("  float4 zr[ZPT];", "  if (N > 0) return;\n  float4 zr[ZPT];")],
    # the same with a 1 KB LDS allocation (the launch floor without the 156 KB workgroup LDS)
    "emptysmall": [("  float4 zr[ZPT];", "  if (N > 0) return;\n  float4 zr[ZPT];"),
                   ("  __shared__ __attribute__((aligned(16))) float smem[L::TOTAL];",
                    "  __shared__ __attribute__((aligned(16))) float smem[256];")],
    # no code-count atomics
    "nohist": [("    if (c != 0.f) atomicAdd(counts + tid, c);", "    if (c == -1.f) atomicAdd(counts + tid, c);")],
}


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "base"
    src = open(os.path.join(CSRC, "vq.hip")).read()
    start = src.index("void vq_fwd_pinned_kernel(")
    head, body = src[:start], src[start:]
    for anchor, n, how in ANCHORS:
        i = body.find(anchor)
        if i < 0:
            sys.exit(f"anchor for stamp {n} not found: {anchor[:50]!r}")
        st = "".join("  " + (RTIME if k >= 8 else STAMP).format(n=k) + "\n" for k in n)
        if how == "before":
            body = body[:i] + st + body[i:]
        elif how == "after":
            j = body.index("\n", i) + 1
            body = body[:j] + st + body[j:]
        else:
            j = i + len(anchor) - 1
            body = body[:j] + st + body[j:]
    for a, b in VARIANTS[variant]:   # inside the pinned kernel (and below it) only, after the stamps
        i = body.find(a)
        if i < 0:
            sys.exit(f"variant {variant}: text not found: {a[:50]!r}")
        body = body[:i] + b + body[i + len(a):]
    ns = head.index("namespace {")
    head = head[:ns] + "__device__ unsigned long long vq_stamp_buf[256 * 8 * 16];\n" + head[ns:]
    tail = ('\nextern "C" void vq_probe_stamps(unsigned long long* out) {\n'
            "  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(vq_stamp_buf), sizeof(vq_stamp_buf));\n}\n")
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, f"vq_stamped_{variant}.hip")
    open(path, "w").write(head + body + tail)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
           "-I", CSRC, path, os.path.join(CSRC, "runtime.hip"), "-o", os.path.join(OUT, "vqs.so" if variant == "base" else f"vqs_{variant}.so")]
    subprocess.check_call(cmd)
    print("built", cmd[-1])


if __name__ == "__main__":
    main()
