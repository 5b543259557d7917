"""Build tools/probe/build/vqs.so: a probe copy of csrc/vq.hip whose codebook-pinned forward writes s_memtime stamps
at its phase boundaries (thread 0 of the first 256 workgroups, vector stores into a __device__ buffer), plus
`vq_probe_stamps(uint64_t out[256 * 8])`.  The product source carries no probe code; the stamps are spliced in here
at fixed anchors (the build fails if one is missing).  Read by tools/probe/vq_stamps_probe.py on the GPU box.
usage (CPU side): python tools/probe/vq_stamps_build.py"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "vq-vae-transformer-arc-welding_amd", "csrc")
OUT = os.path.join(HERE, "build")

STAMP = "if (threadIdx.x == 0 && blockIdx.x < 256) vq_stamp_buf[blockIdx.x * 8 + {n}] = __builtin_amdgcn_s_memtime();"

# (anchor text inside vq_fwd_pinned_kernel, stamp index, insert before (False) / after (True) the anchor)
ANCHORS = [
    ("  const int64_t row0 = (int64_t)blockIdx.x * ROWS;\n\n  // ---- the codebook: float4", 0, "mid"),
    ("  __syncthreads();\n  // ---- |z|^2 per row and |e_k|^2 per code", 1, "mid"),
    ("  // software-pipelined LDS reads", 2, "before"),
    ("  // ---- distances and this lane's (d, k) minimum", 3, "before"),
    ("  __syncthreads();   // every wave's codebook reads are done", 4, "after_line"),
    ("                    counts, sqerr, zq2, zq2_bf16);\n}", 5, "before_brace"),
]


def main():
    src = open(os.path.join(CSRC, "vq.hip")).read()
    start = src.index("void vq_fwd_pinned_kernel(")
    head, body = src[:start], src[start:]
    for anchor, n, how in ANCHORS:
        i = body.find(anchor)
        if i < 0:
            sys.exit(f"anchor for stamp {n} not found: {anchor[:50]!r}")
        st = "  " + STAMP.format(n=n) + "\n"
        if how == "before":
            body = body[:i] + st + body[i:]
        elif how == "mid":   # after the first line of the anchor
            j = body.index("\n", i) + 1
            body = body[:j] + st + body[j:]
        elif how == "after_line":
            j = body.index("\n", i) + 1
            body = body[:j] + st + body[j:]
        elif how == "before_brace":
            j = i + len(anchor) - 1
            body = body[:j] + st + body[j:]
    ns = head.index("namespace {")
    head = head[:ns] + "__device__ unsigned long long vq_stamp_buf[256 * 8];\n" + head[ns:]
    tail = ('\nextern "C" void vq_probe_stamps(unsigned long long* out) {\n'
            "  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(vq_stamp_buf), sizeof(vq_stamp_buf));\n}\n")
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, "vq_stamped.hip")
    open(path, "w").write(head + body + tail)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-shared",
           "-I", CSRC, path, os.path.join(CSRC, "runtime.hip"), "-o", os.path.join(OUT, "vqs.so")]
    subprocess.check_call(cmd)
    print("built", os.path.join(OUT, "vqs.so"))


if __name__ == "__main__":
    main()
