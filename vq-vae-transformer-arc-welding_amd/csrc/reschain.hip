// Fused ResBlock chains of the bf16 VQ-VAE step: the encoder's and the decoder's ResBlock stacks
// (model/vq_vae_patch_embedd.py:60-74 ResBlock inside CNNBlock :103-110), each as ONE persistent launch per direction.
//   forward   h = conv1(a) + b1,  a1 = GELU(h),  x' = x + Dropout(conv2(a1) + b2),  a' = GELU(x')      (a = GELU(x))
//   backward  gh = conv2^T(go) * GELU'(h),  gx = gx' + conv1^T(gh) * GELU'(x),  go = gx * mask(block r-1)
// The forward saves GELU'(h) and GELU'(x') (bf16) for the backward, evaluated from the same Phi / exp as the GELU it
// computes anyway (two VALU operations more per element); the backward multiplies by them and evaluates no
// transcendental (only GELU'(x_0) of the stack input, for block 0's conv1, is its own).  Same-bytes as saving h and x'.
// Encoder (CNNBlock(seperate=True)): each conv sees a length-1 token slice, so it is its centre tap, a [H][H]
// contraction per token (TAPS = 1).  Decoder (seperate=False): k = 3, padding-1 convs along each 16-token window
// (TAPS = 3, K = 3H: tap j reads token t + j - 1 forward, t - j + 1 backward, zero outside the window).  Either way a
// 64-token row block (four whole windows) is self-contained through all R blocks.  The unfused path runs each conv as
// its own GEMM launch (2R launches per direction).  Here one launch walks a row block through
// all 2R convs:
//  * one 512-thread workgroup per CU (N / 64 of them: 256 at configs[1]); wave w owns output channels
//    [64 w, 64 w + 64) of every conv, so each weight element is read by exactly one wave of a workgroup: the
//    weights go global -> VGPRs directly (no LDS staging), two K steps ahead, and the stream runs on across conv
//    boundaries (weights never depend on activations).  The weights are read from fragment-packed copies
//    (aw_res_pack_weights): every wave load instruction is one contiguous KB.  Read in the [out][in] layout (16 rows
//    x 64 B per instruction) the same loop ran its K steps 2.3x slower (22 k vs 9.5 k cycles per conv, probe
//    stamps): each 128-B line was fetched twice, once per half;
//  * the row block's activations never leave the CU between convs: two LDS images [token][channel] (bf16, 16-B
//    chunks XOR-swizzled by token: conflict-free ds_read_b128 fragments), one read by the current conv, the other
//    written by its epilogue as the next conv's operand.  The decoder's images hold a zero row before and after each
//    16-token window (69 rows): a shifted tap's fragment read at a window edge lands on it, so the padding costs no
//    instruction;
//  * no workgroup barrier between convs: wave w publishes its 64-channel slice of the next image with an LDS flag,
//    and a K step of the next conv waits only for the slice it reads (K steps 2w', 2w' + 1 of the first tap = wave
//    w''s slice).  The waves drift apart, so one wave's epilogue (VALU, stores) runs under its SIMD partner's MFMAs
//    (an initial half-conv delay of waves 4-7 helped an earlier form of the epilogues by 10 %; with the early
//    publish and line-loaded pre-activations it costs 2-5 %, so all waves start together).
//    The image ring stays safe: a wave writing image (c + 2) & 1 in conv c + 1's epilogue has read all of conv c's
//    slices, so every wave is past conv c's K loop (the one that read that image);
//  * the product is computed transposed, C^T = W X^T (v_mfma_f32_16x16x32_bf16, A = weight rows, B = tokens), so a
//    lane's accumulator holds 4 CONSECUTIVE channels of one token: LDS writes, residual and pre-activation reads are
//    8-B pieces, and the dropout mask costs one hash per 4 elements exactly as in the unfused epilogue
//    (aw_dropout_scale4 on the group row*H + c, c % 4 == 0).  The forward hashes block r's mask inside its conv2 K
//    loop (VALU under the MFMAs) and stores the keep bits for the backward;
//  * global stores are whole 128-B lines (a wave's 64 channels of 8 tokens per instruction), read back from LDS:
//    the output that is also the next operand from the wave's own slice of the next image, the other one through a
//    2 KB per-wave scratch.  Stored straight from the accumulator layout (32-B pieces per token) they cost 20 k
//    cycles per epilogue (probe stamps);
//  * the residual stream (x forward, gx backward) stays in registers as bf16 (the bf16 mode's resid dtype); the
//    weight gradients' operands are written as the unfused path writes them (a1, a forward; gh and the masked gx
//    backward), and in place of the unfused path's h and x the forward saves GELU'(h), GELU'(x') for the backward.
// Per element the epilogues run the unfused GEMM epilogue's operations in its order (gemm_core.h), and each
// accumulator sees the same MFMA sequence (K ascending in 32-deep steps, tap-major as the implicit conv GEMM), so
// the forward's outputs a1 / a / keep bits are the unfused path's bit for bit; the saved derivatives are GELU' of the
// f32 pre-activation (the unfused backward: of its bf16 copy) rounded to bf16, so the backward tracks the unfused one
// to bf16 rounding (tests/test_res_chain.py).
#include "common.h"

#include <type_traits>

#pragma clang diagnostic ignored "-Winline-asm"

// (Probe builds with parts left out are made from text replacements of this file: tools/probe/res_chain_variants.py.)

namespace {

constexpr int EC_H = 512;                   // channels (the reference's hidden_dim)
constexpr int EC_ROWS = 64;                 // tokens per workgroup
constexpr int EC_NTH = 512;                 // 8 waves x 64 output channels
constexpr int EC_ROWB = EC_H * 2;           // bytes per image row (bf16)
constexpr int EC_SCR = 2048;                // per-wave scratch: 16 tokens x 64 channels bf16, [token][128 B]
constexpr int EC_SEG = 16;                  // decoder window (tokens), one 16-token fragment group

// LDS / weight geometry of a chain with TAPS taps per conv
template <int TAPS> struct EcGeo {
  static constexpr int KS = 16 * TAPS;                             // 32-deep K steps per conv
  static constexpr int JS = (TAPS == 1 ? 16 : 17) * EC_ROWB;       // image offset of 16-token group j + 1 vs j
  static constexpr int R0 = TAPS == 1 ? 0 : EC_ROWB;               // image offset of token 0 (zero row ahead)
  static constexpr int IMG = (TAPS == 1 ? 64 : 69) * EC_ROWB;      // one activation image
  static constexpr int SCR = 2 * IMG;                              // per-wave scratch
  static constexpr int FLAGS = SCR + 8 * EC_SCR;                   // 8 per-wave "epilogues done" counters
  static constexpr int BIAS = FLAGS + 64;                          // per-wave bias slot (the current conv's 64)
  static constexpr int LDS = BIAS + 8 * 256;
  static constexpr uint32_t WBYTES = (uint32_t)EC_H * EC_H * 2 * TAPS;   // one packed weight matrix
  static constexpr int WWAVE = 4 * KS * 1024;                      // a wave's 4 packed block rows
  // Image swizzle key of token u of a 16-token group: chunk c of the token sits at chunk c ^ key(u).  Three kinds of
  // LDS access see the keys: the B-fragment reads of the K loop (the decoder's shifted taps read rows u - 1 / u + 1
  // beside u: with key = u the 16 lanes of a ds_read_b128 group hit one bank slot twice under either shift, 38 % of
  // the decoder chain's LDS cycles were bank conflicts), the epilogue's ds_write_b64 (at best two lanes per bank) and
  // the store path's whole-line slice reads (EcStore::ir, eight tokens x eight chunks per instruction: the identity and
  // the round-5 decoder keys put two lanes of a group on one slot there, 21-23 % conflicts in the encoder chains).
  // Both tables come from an exhaustive search over all three (tools/probe/chain_swizzle.py; the encoder's only for the
  // unshifted reads it makes).  The zero rows ahead of / behind a window (u = -1 / 16) read with keys 15 / 0.
  static constexpr uint64_t KEYS = TAPS == 1 ? 0xfe76dc54ba329810ull : 0xf53ac739685ace10ull;
  __device__ static int key(int u) { return u < 0 ? 15 : u > 15 ? 0 : (int)((KEYS >> (4 * u)) & 15); }
};
static_assert(EcGeo<3>::LDS <= 160 * 1024, "decoder chain LDS");

typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t ec_rsrc(const void* p, uint32_t nbytes) {
  // a NULL output gets a zero-record descriptor: every store through it is dropped
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, p ? nbytes : 0u, 0x00020000);
}
// Global accesses are buffer instructions: the lane's offset in a VGPR, the compile-time part (tile row / column
// block) in the SGPR soffset.  Folded into the VGPR offset (the buffer immediate holds only 12 bits) each constant
// became a VGPR of its own, held across the whole kernel: 25 extra VGPRs and the spills that came with them.
__device__ __forceinline__ u32x2 ec_load8(rsrc_t r, uint32_t voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
}
// Store-data hazard: a VMEM store of more than 64 bits of data reads its data VGPRs after issue, so a VALU write of
// those VGPRs needs 2 wait states behind it on gfx94x / gfx950 (LLVM GCNHazardRecognizer: VALUWaitStates = 2;
// cdna_hip_programming.md 5.7 item 1).  ROCm 7.2's hazard recognizer pads it for every form EXCEPT a MUBUF / MTBUF
// store whose soffset is a register (createsVALUHazard skips those, the SI-era premise that the hazard needs an
// immediate soffset), and these stores pass the tile offset in an SGPR soffset.  Without a pad the compiler emitted
//   buffer_store_dwordx4 v[34:37], v217, s[24:27], s65 offen sc1
//   v_add_u32_e32 v34, 0xc008, v222          ; the next LDS address, 0 wait states later
// and on the GPU the stored line's first dword intermittently came out as that address (round 5).  The pad: one
// s_nop 1 (2 wait states) that names the data registers, so none of them is reused before it.  Audited over the
// whole library's ISA by tests/test_isa_hazards.py.
template <bool WT> __device__ __forceinline__ void ec_store16(rsrc_t r, uint32_t voff, int soff, uint4 v) {
  aw_v4i32 u;
  memcpy(&u, &v, 16);
  // sc1 (write-through) or nt: the lines must not stay in the XCD's L2, which holds the weight stream
  __builtin_amdgcn_raw_buffer_store_b128(u, r, voff, soff, WT ? 16 : 2);
  asm volatile("s_nop 1" ::"v"(u));
}
// 64-bit data: outside the hazard (and soffset 0, which the compiler pads anyway)
__device__ __forceinline__ void ec_store8(rsrc_t r, uint32_t voff, u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, 0, 2);
}
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
// 4 floats -> 4 bf16 (round to nearest even, as the unfused epilogue's (bf16) casts): two v_cvt_pk_bf16_f32 (the
// element-wise casts compiled to a cvt per element plus byte shuffles)
__device__ __forceinline__ u32x2 ec_pack(const float (&v)[4]) {
  const bf16x2 lo = __builtin_convertvector((f32x2){v[0], v[1]}, bf16x2);
  const bf16x2 hi = __builtin_convertvector((f32x2){v[2], v[3]}, bf16x2);
  return u32x2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}
__device__ __forceinline__ void ec_unpack(u32x2 u, float (&v)[4]) {
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xFFFF0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xFFFF0000u);
}
__device__ __forceinline__ uint4 ec_wload(rsrc_t r, int voff, int soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  uint4 u;
  memcpy(&u, &v, 16);
  return u;
}
__device__ __forceinline__ void ec_lds_w8(char* smem, int off, u32x2 v) { *reinterpret_cast<u32x2*>(smem + off) = v; }
__device__ __forceinline__ uint4 ec_lds_r16(const char* smem, int off) {
  return *reinterpret_cast<const uint4*>(smem + off);
}

// image [token][k]: 16-B chunk c of token t (16-token group j, t % 16 = u) sits at R0 + j JS + u ROWB, chunk
// c ^ key(u) (EcGeo::key).  A fragment read (lane: token u + tap shift, chunk 4s + g) hits 16 distinct 16-B bank slots
// in each ds_read_b128 lane group.  The decoder's zero rows (at j JS, j = 0..4) are read by the shifted taps only.
template <class G> __device__ __forceinline__ int ec_off(int tok, int chunk) {
  return G::R0 + (tok >> 4) * G::JS + (tok & 15) * EC_ROWB + ((chunk ^ G::key(tok & 15)) << 4);
}

// The first operand image of a chain: rows [row0, row0 + 64) of a [N][H] bf16 tensor (zeros past N); the decoder
// images' zero rows are cleared here and never written again.
template <class G>
__device__ __forceinline__ void ec_load_image(char* img, const void* src, int64_t row0, uint32_t nbytes, int tid) {
  const rsrc_t rs = ec_rsrc(src, nbytes);
#pragma unroll
  for (int q = 0; q < (EC_ROWS * EC_ROWB / 16) / EC_NTH; ++q) {
    const int c = tid + q * EC_NTH, tok = c >> 6, ch = c & 63;
    const uint32_t off = (uint32_t)((row0 + tok) * EC_ROWB + ch * 16);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    uint4 u;
    memcpy(&u, &v, 16);
    *reinterpret_cast<uint4*>(img + ec_off<G>(tok, ch)) = u;
  }
  if constexpr (G::R0 != 0) {
    for (int c = tid; c < 2 * 5 * 64; c += EC_NTH) {   // 2 images x 5 zero rows x 64 chunks
      const int im = c / 320, row = (c % 320) >> 6, ch = c & 63;
      *reinterpret_cast<uint4*>(img + im * G::IMG + row * G::JS + ch * 16) = uint4{0u, 0u, 0u, 0u};
    }
  }
}

// ---------------------------------------------------------------- inter-wave hand-off through LDS
typedef __attribute__((address_space(3))) volatile int lds_vint;
template <class G> __device__ __forceinline__ lds_vint* ec_flag(char* smem, int wv) {
  // an LDS pointer (ds_read / ds_write): through a generic pointer the flags compiled to flat accesses
  return (lds_vint*)(smem + G::FLAGS) + wv;
}
// wait until wave wv has published `target` epilogues (its slice of the image this conv reads is written)
template <class G> __device__ __forceinline__ void ec_wait(char* smem, int wv, int target) {
  while (__builtin_amdgcn_readfirstlane(*ec_flag<G>(smem, wv)) < target) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");   // the image reads that follow stay behind the flag read
}
// publish this wave's slice of the next image (every LDS write of it performed first)
template <class G> __device__ __forceinline__ void ec_publish(char* smem, int w, int lane, int count) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) *ec_flag<G>(smem, w) = count;
}

// One epilogue scheduling region per fragment: bounded live ranges (regions of 2, 4 or 16 fragments, letting the
// scheduler interleave their VALU chains, measured within 1-3 %: the epilogue is bound by its VALU issue, not by
// dependency latency).
__device__ __forceinline__ void ec_frag_fence(int) { __builtin_amdgcn_sched_barrier(0); }

// GELU / GELU' of a fragment's 4 values, element by element (the same operations as aw_gelu4 / aw_gelu_grad4, so
// the same bits as the unfused GEMM epilogues): written per element, the compiler packs only where it pays (the
// fully packed pair form measured 3 % slower here, MI355X_MICROARCH.md: packed f32 VALU beside MFMAs)
__device__ __forceinline__ void ec_gelu_grad4(const float (&v)[4], float (&y)[4]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) y[e] = gelu_erf_grad_fast(v[e]);
}
// both from one Phi / exp evaluation: y = GELU(v) with ec_gelu4's bits, d = GELU'(v) with ec_gelu_grad4's
__device__ __forceinline__ void ec_gelu_and_grad4(const float (&v)[4], float (&y)[4], float (&d)[4]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float ex;
    const float phi = aw_phi_e(v[e], ex);
    y[e] = v[e] * phi;
    d[e] = fmaf(v[e] * AW_INV_SQRT2PI, ex, phi);
  }
}

// Weight fragment (i, s) of wave w (rows 64w + 16i .. +15, k 32s .. 32s + 31) in the fragment-packed layout: block
// (4w + i, s) is one KB, lane l's 16 B at 16 l (aw_res_pack_weights).
template <class G> __device__ __forceinline__ constexpr int ec_woff(int i, int s) { return (i * G::KS + s) * 1024; }

// Dropout keep bits of a lane's 16 fragments (aw_res_dropout_masks): fragment f = 4i + j, bit 4 (f & 7) + e of word
// f >> 3 = element e is kept.  Word ((r * nwg + wg) * 512 + tid) of the mask buffer.
__device__ __forceinline__ size_t ec_keep_idx(int r, int tid) {
  return ((size_t)r * gridDim.x + blockIdx.x) * EC_NTH + tid;
}
__device__ __forceinline__ u32x2 ec_keep(const uint64_t* masks, int r, int tid) {
  return __builtin_bit_cast(u32x2, masks[ec_keep_idx(r, tid)]);
}
// the keep bits of fragment f = 4i + j of the lane with token row `row` (16 j added) and channels c0 (+ 16 i) ..
// + 3: aw_gemm's epilogue hash of group (row * H + c) / 4 under `seed`
__device__ __forceinline__ uint32_t ec_keep_bits(uint64_t seed, uint64_t grp0, int f, uint32_t thr) {
  // opaque group: (g + 1) * golden does not depend on the conv, and hoisted out of the conv loop the 16 products
  // held 32 VGPRs through the whole kernel (and spilled)
  uint32_t lo = (uint32_t)grp0, hi = (uint32_t)(grp0 >> 32);
  asm volatile("" : "+v"(lo), "+v"(hi));
  const uint64_t h = aw_hash_group(seed, (((uint64_t)hi << 32) | lo) + 2048u * (f & 3) + 4u * (f >> 2));
  uint32_t k = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) k |= (((uint32_t)(h >> (16 * e)) & 0xFFFFu) >= thr ? 1u : 0u) << (4 * (f & 7) + e);
  return k;
}
__device__ __forceinline__ void ec_scales(u32x2 keep, int i, int j, float k, float (&ds)[4]) {
  const int f = 4 * i + j;
  const uint32_t b = ((f >> 3) ? keep.y : keep.x) >> (4 * (f & 7));
#pragma unroll
  for (int e = 0; e < 4; ++e) ds[e] = (b >> e) & 1u ? k : 0.f;
}

// One conv: acc[i][j] (channels 64w + 16i + 4g .. +3 of token 16j + li) = sum over the TAPS x 512 inputs, K
// ascending in 32-deep steps (tap-major).  wf[s & 1] holds the weight fragments of step s on entry; the loads of step
// s + 2 are issued behind step s's MFMAs (into the same registers), those of the last two steps' successors from
// the next conv's weights (rn, when has_next).  Image reads of step s = 16 t + 4a + b (tap t): token 16j + li + d_t,
// chunk 4(4a + b) + g lives at (rb[t] ^ 64 b) + 256 a + JS j + io.  Step 2v of tap 0 waits for flag v >= target
// (another wave's slice).  step(s) runs behind step s's MFMAs, tail() behind the last K step's weight loads.
template <class G, typename Tail, typename Step>
__device__ __forceinline__ void ec_conv(f32x4 (&acc)[4][4], uint4 (&wf)[2][4], char* smem, const int (&rb)[G::KS / 16],
                                        int io, rsrc_t rc, rsrc_t rn, bool has_next, int wl, int w, int target,
                                        Tail tail, Step step) {
  constexpr int T = G::KS / 16;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int rbi[T];
#pragma unroll
  for (int t = 0; t < T; ++t) rbi[t] = rb[t] + io;
#pragma unroll
  for (int s = 0; s < G::KS; ++s) {
    const int t = s >> 4, kk = s & 15;
    // image fragments of step s (a wave's partner on the SIMD covers their latency): read at the step, not one
    // ahead -- the 16 registers of a second set made the masked (dropout) kernels spill
    if (t == 0 && (kk & 1) == 0 && (kk >> 1) != w) ec_wait<G>(smem, kk >> 1, target);
    uint4 bf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = ec_lds_r16(smem, (rbi[t] ^ (64 * (kk & 3))) + (kk >> 2) * 256 + j * G::JS);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[s & 1][i]),
                                                            __builtin_bit_cast(bf16x8, bf[j]), acc[i][j], 0, 0, 0);
    if (s + 2 < G::KS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) wf[s & 1][i] = ec_wload(rc, wl, ec_woff<G>(i, s + 2));
    } else if (has_next) {
#pragma unroll
      for (int i = 0; i < 4; ++i) wf[s & 1][i] = ec_wload(rn, wl, ec_woff<G>(i, s + 2 - G::KS));
    }
    step(s);
    if (s == G::KS - 1) tail();
    // one scheduling region per K step: the prefetch stays two steps ahead (left alone, the scheduler sinks each
    // load down to its MFMA and waits for it there)
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Per-lane constants of the chain kernels.  Fragment (i, j) of a lane covers token 16j + li and channels
// 64w + 16i + 4g .. +3; its image position is wb[i] + JS j (plus the image offset).  DIR: +1 forward (tap t reads
// token + t - 1), -1 backward (token - t + 1).
template <class G, int DIR> struct EcLane {
  static constexpr int T = G::KS / 16;
  int lane, li, g, w;
  int wl;        // weight lane offset in a packed matrix: block (4w, 0), lane l
  int rb[T];     // image read base of tap t, b = 0; b's is rb ^ 64 b (the swizzle moves bits 6-7 only)
  int wb0;       // image write base of i = 0; i's is wb0 ^ 32 i
  __device__ __forceinline__ EcLane(int tid) {
    lane = tid & 63;
    w = tid >> 6, g = lane >> 4, li = lane & 15;
    wl = w * G::WWAVE + lane * 16;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int tp = li + (T == 1 ? 0 : DIR * (t - 1)), key = G::key(tp);   // tp = -1 / 16: the zero rows
      rb[t] = G::R0 + tp * EC_ROWB + ((4 * (key >> 2) + (g ^ (key & 3))) << 4);
    }
    wb0 = G::R0 + li * EC_ROWB + (((8 * w + (g >> 1)) ^ G::key(li)) << 4) + (g & 1) * 8;
  }
  __device__ __forceinline__ int wb(int i) const { return wb0 ^ (32 * i); }
};
// The store side, derived in the epilogue (not held across the K loop).  Global stores write a wave's 64-channel
// slice (128 B per token) of 8 tokens per instruction, lane -> (token lane >> 3, 16-B chunk lane & 7), at gs + 8192 q
// for tokens 8q .. 8q + 7.  The slice comes from the wave's own chunks of the next image (ir[q & 1] + JS (q >> 1))
// or from its scratch (16 tokens at a time: written at sw[i], read at sr[q]; the 16-B chunk of token t XOR-swizzled
// by t >> 1, so that a ds_write_b64 of the fragment layout puts each lane on a bank of its own -- with t & 7 tokens t
// and t + 8 met on one bank -- and the line-layout ds_read_b128 / ds_write_b128 groups stay conflict-free).
template <class G> struct EcStore {
  int ir[2];     // image own-slice read bases (q parity), without the image offset
  int sw[4];     // scratch write bases per i
  int sr;        // scratch line base of tokens lane >> 3; tokens 8 + (lane >> 3) at srq(1) = (sr ^ 64) + 1024
  __device__ __forceinline__ int srq(int q) const { return q ? (sr ^ 64) + 1024 : sr; }
  uint32_t gs;   // global byte offset of this lane's store piece for tokens 0..7
  __device__ __forceinline__ EcStore(int tid, int64_t row0) {
    const int lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
    const int t8 = lane >> 3, c8 = lane & 7;
#pragma unroll
    for (int p = 0; p < 2; ++p) ir[p] = G::R0 + (8 * p + t8) * EC_ROWB + (((8 * w + c8) ^ G::key(8 * p + t8)) << 4);
    const int sbase = G::SCR + w * EC_SCR;
#pragma unroll
    for (int i = 0; i < 4; ++i) sw[i] = sbase + li * 128 + (((2 * i + (g >> 1)) ^ (li >> 1)) << 4) + (g & 1) * 8;
    sr = sbase + t8 * 128 + ((c8 ^ (t8 >> 1)) << 4);   // (t8 + 8) >> 1 = (t8 >> 1) ^ 4: chunk bit 2, byte bit 6
    gs = (uint32_t)(((row0 + t8) * EC_H + 64 * w + 8 * c8) * 2);
  }
};

// 16 fragments' worth of 8-B pieces of a [N][H] bf16 tensor
__device__ __forceinline__ void ec_load_frags(u32x2 (&d)[4][4], rsrc_t r, uint32_t go) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) d[i][j] = ec_load8(r, go, 16384 * j + 32 * i);
}
__device__ __forceinline__ uint32_t ec_frag_off(int64_t row0, int li, int w, int g) {
  return (uint32_t)(((row0 + li) * EC_H + 64 * w + 4 * g) * 2);
}
// the wave's own 64-channel slice of all 64 tokens of an image -> global, as whole lines
template <class G, bool WT>
__device__ __forceinline__ void ec_store_slice(const char* smem, int img, const EcStore<G>& S, rsrc_t r) {
  const int b0 = img + S.ir[0], b1 = img + S.ir[1];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    ec_store16<WT>(r, S.gs, 8192 * q, ec_lds_r16(smem, ((q & 1) ? b1 : b0) + G::JS * (q >> 1)));
}
// the wave's scratch (tokens 16 j .. 16 j + 15 of its slice) -> global
template <class G, bool WT>
__device__ __forceinline__ void ec_store_scratch(const char* smem, int j, const EcStore<G>& S, rsrc_t r) {
#pragma unroll
  for (int q = 0; q < 2; ++q) ec_store16<WT>(r, S.gs, 8192 * (2 * j + q), ec_lds_r16(smem, S.srq(q)));
}

template <class G> __device__ __forceinline__ void ec_init(char* smem, int tid) {
  if (tid < 8) *ec_flag<G>(smem, tid) = 0;
}

template <int TAPS, bool DROP, bool WT>
__global__ __launch_bounds__(EC_NTH) void res_chain_fwd_kernel(aw_res_chain_fwd_args P) {
  using G = EcGeo<TAPS>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * EC_ROWS;
  const EcLane<G, 1> L(tid);
  const uint32_t nbytes = (uint32_t)(P.N * EC_ROWB);
  const int R = P.R, NC = 2 * R;

  ec_init<G>(smem, tid);
  ec_load_image<G>(smem, P.a0, row0, nbytes, tid);
  u32x2 xr[4][4];   // the residual stream x (bf16) of this lane's fragments, kept in registers through the chain
  ec_load_frags(xr, ec_rsrc(P.x0, nbytes), ec_frag_off(row0, L.li, L.w, L.g));
  uint4 wf[2][4];
  {
    const rsrc_t r0 = ec_rsrc(P.w1[0], G::WBYTES);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wf[0][i] = ec_wload(r0, L.wl, ec_woff<G>(i, 0));
      wf[1][i] = ec_wload(r0, L.wl, ec_woff<G>(i, 1));
    }
  }
  const rsrc_t rmask = ec_rsrc(DROP ? P.drop_masks : nullptr, (uint32_t)(R * gridDim.x * EC_NTH * 8));
  const uint32_t thr = aw_drop_threshold(P.drop_p);
  // dropout group of fragment (0, 0): (row * H + c) / 4 for token row0 + li, channel 64w + 4g
  const uint64_t grp0 = (uint64_t)(row0 + L.li) * (EC_H / 4) + 16 * L.w + L.g;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  for (int c = 0; c < NC; ++c) {
    const int r = c >> 1;
    const bool second = (c & 1) != 0;
    const rsrc_t rc = ec_rsrc(second ? P.w2[r] : P.w1[r], G::WBYTES);
    const bool has_next = c + 1 < NC;
    const rsrc_t rn = ec_rsrc(has_next ? (second ? P.w1[r + 1] : P.w2[r]) : nullptr, G::WBYTES);
    const int io = (c & 1) * G::IMG, no = ((c + 1) & 1) * G::IMG;
    f32x4 acc[4][4];
    // this conv's bias, one value per lane (the wave's 64 channels), loaded ahead of the K loop and parked in the
    // wave's LDS slot at its end (read in the epilogue as a 16-B broadcast per fragment row: no L2 latency there)
    const float bias_l = (second ? P.b2[r] : P.b1[r])[64 * L.w + L.lane];
    // block r's dropout keep bits, hashed one fragment per K step of conv2 (VALU under the MFMAs) and stored for the
    // backward behind the last K step
    const uint64_t seed = DROP && second ? aw_seed_mix(P.drop_seed[r], P.seed_ptr) : 0;
    uint32_t kb[2] = {0u, 0u};
    auto hash = [&](int s) {
      if (DROP && second && s < 16) kb[s >> 3] |= ec_keep_bits(seed, grp0, s, thr);
    };
    auto park = [&] {
      *reinterpret_cast<float*>(smem + G::BIAS + 256 * L.w + 4 * L.lane) = bias_l;
      if (DROP && second) ec_store8(rmask, (uint32_t)(ec_keep_idx(r, tid) * 8), u32x2{kb[0], kb[1]});
    };
    ec_conv<G>(acc, wf, smem, L.rb, io, rc, rn, has_next, L.wl, L.w, c, park, hash);
    const u32x2 keep = {kb[0], kb[1]};
    int nwb[4];   // this lane's write positions in the next image (fragment i; + JS j)
#pragma unroll
    for (int i = 0; i < 4; ++i) nwb[i] = L.wb(i) + no;

    auto bias = [&](int i, float (&bv)[4]) {   // channels 64w + 16i + 4g .. +3 from the wave's LDS slot
      const float4 b4 = *reinterpret_cast<const float4*>(smem + G::BIAS + 256 * L.w + 64 * i + 16 * L.g);
      bv[0] = b4.x, bv[1] = b4.y, bv[2] = b4.z, bv[3] = b4.w;
    };
    const EcStore<G> S(tid, row0);
    // The slice is published as soon as the next operand image holds it (the other waves' next K loops wait for
    // it); the saved tensor that goes through the scratch (h, x') follows the publish.
    if (!second) {
      // a1 = GELU(h), h = conv1 + b1: a1 into the next operand image (stored from there once published); GELU'(h)
      // from the same Phi into the scratch, saved 16 tokens at a time (held in registers until after the publish, the
      // 32 VGPRs made the kernel spill 145-175)
      const rsrc_t rh = ec_rsrc(P.dgelu_h[r], nbytes);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v[4], y[4], d[4], bv[4];
          bias(i, bv);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
          ec_gelu_and_grad4(v, y, d);
          ec_lds_w8(smem, nwb[i] + G::JS * j, ec_pack(y));
          ec_lds_w8(smem, S.sw[i], ec_pack(d));
          ec_frag_fence(4 * j + i);
        }
        ec_store_scratch<G, WT>(smem, j, S, rh);
        __builtin_amdgcn_sched_barrier(0);
      }
      ec_publish<G>(smem, L.w, L.lane, c + 1);
      ec_store_slice<G, WT>(smem, no, S, ec_rsrc(P.a1[r], nbytes));
    } else {
      // x' = x + Dropout(conv2 + b2) (kept in registers) and a' = GELU(x') (the next operand image), GELU'(x') saved
      // through the scratch; the last block stores x_R itself (the next stage's operand), staged in the image
      const bool last = r == R - 1;
      const float dk = DROP ? 1.f / (1.f - P.drop_p) : 1.f;
      auto resid = [&](int i, int j, float (&v)[4]) {
        float ds[4] = {1.f, 1.f, 1.f, 1.f}, xv[4], bv[4];
        bias(i, bv);
        if constexpr (DROP) ec_scales(keep, i, j, dk, ds);
        ec_unpack(xr[i][j], xv);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = aw_epi_mad(acc[i][j][e] + bv[e], ds[e], DROP, xv[e], true);
        xr[i][j] = ec_pack(v);
      };
      if (!last) {
        const rsrc_t rx = ec_rsrc(P.dgelu_x[r], nbytes);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v[4], y[4], d[4];
            resid(i, j, v);
            ec_gelu_and_grad4(v, y, d);
            ec_lds_w8(smem, nwb[i] + G::JS * j, ec_pack(y));
            ec_lds_w8(smem, S.sw[i], ec_pack(d));
            ec_frag_fence(4 * j + i);
          }
          ec_store_scratch<G, WT>(smem, j, S, rx);
          __builtin_amdgcn_sched_barrier(0);
        }
        ec_publish<G>(smem, L.w, L.lane, c + 1);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v[4];
            resid(i, j, v);
            ec_lds_w8(smem, nwb[i] + G::JS * j, xr[i][j]);
            ec_frag_fence(4 * i + j);
          }
      }
      ec_store_slice<G, WT>(smem, no, S, ec_rsrc(P.a[r], nbytes));
    }
  }
}

template <int TAPS, bool DROP, bool WT>
__global__ __launch_bounds__(EC_NTH) void res_chain_bwd_kernel(aw_res_chain_bwd_args P) {
  using G = EcGeo<TAPS>;
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * EC_ROWS;
  const EcLane<G, -1> L(tid);
  const uint32_t nbytes = (uint32_t)(P.N * EC_ROWB);
  const int R = P.R, NC = 2 * R;
  const uint32_t fo = ec_frag_off(row0, L.li, L.w, L.g);

  ec_init<G>(smem, tid);
  ec_load_image<G>(smem, P.gxo, row0, nbytes, tid);
  u32x2 gr[4][4];   // the residual gradient dL/dx (bf16), kept in registers through the chain
  ec_load_frags(gr, ec_rsrc(P.gx, nbytes), fo);
  uint4 wf[2][4];
  {
    const rsrc_t r0 = ec_rsrc(P.w2t[R - 1], G::WBYTES);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wf[0][i] = ec_wload(r0, L.wl, ec_woff<G>(i, 0));
      wf[1][i] = ec_wload(r0, L.wl, ec_woff<G>(i, 1));
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  for (int c = 0; c < NC; ++c) {
    const int r = R - 1 - (c >> 1);
    const bool second = (c & 1) != 0;   // false: conv2's input gradient (W2^T), true: conv1's (W1^T)
    const rsrc_t rc = ec_rsrc(second ? P.w1t[r] : P.w2t[r], G::WBYTES);
    const bool has_next = c + 1 < NC;
    const rsrc_t rn = ec_rsrc(has_next ? (second ? P.w2t[r - 1] : P.w1t[r]) : nullptr, G::WBYTES);
    const int io = (c & 1) * G::IMG, no = ((c + 1) & 1) * G::IMG;
    f32x4 acc[4][4];
    // the epilogue's GELU' (the forward's GELU'(h_r) for conv2's gradient, GELU'(x_r) for conv1's; for block 0's
    // conv1 the stack input x_0 itself, whose GELU' is evaluated here) as whole 128-B lines (the wave's 64-channel
    // slice of 8 tokens per load, as the stores), turned into fragments through the wave's scratch in the epilogue;
    // and, for conv1's, block r - 1's dropout keep bits.  Loaded behind the last K step's weight loads:
    // issued earlier, a load would hold up (in vmcnt order) the weight loads issued after it.  Loaded in the
    // fragment layout (16 rows x 32 B per instruction, every line touched by four instructions) the backward ran
    // 40 % slower than with the pre-activations left out (probe), against 7 % for the forward's GELU alone.
    uint4 pl[8];
    u32x2 keep = {0u, 0u};
    auto load_pre = [&] {
      const rsrc_t rp = ec_rsrc(second ? (r > 0 ? P.dgelu_x[r] : P.x0) : P.dgelu_h[r], nbytes);
      const uint32_t gs = (uint32_t)(((row0 + (L.lane >> 3)) * EC_H + 64 * L.w + 8 * (L.lane & 7)) * 2);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, gs, 8192 * q, 0);
        memcpy(&pl[q], &v, 16);
      }
      if (DROP && second && r > 0) keep = ec_keep(P.drop_masks, r - 1, tid);
    };
    ec_conv<G>(acc, wf, smem, L.rb, io, rc, rn, has_next, L.wl, L.w, c, load_pre, [](int) {});
    int nwb[4];   // this lane's write positions in the next image (fragment i; + JS j)
#pragma unroll
    for (int i = 0; i < 4; ++i) nwb[i] = L.wb(i) + no;
    const EcStore<G> S(tid, row0);
    // tokens 16 j .. 16 j + 15 of the pre lines into the scratch (read back below as this lane's fragments (i, j))
    auto stage_pre = [&](int j) {
      *reinterpret_cast<uint4*>(smem + S.srq(0)) = pl[2 * j];
      *reinterpret_cast<uint4*>(smem + S.srq(1)) = pl[2 * j + 1];
    };
    auto pre_frag = [&](int i, float (&pv)[4]) { ec_unpack(*reinterpret_cast<const u32x2*>(smem + S.sw[i]), pv); };

    if (!second) {
      // gh = (W2^T go) * GELU'(h): the next operand image, stored from there (conv1's weight-gradient operand)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stage_pre(j);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float ag[4], v[4];
          pre_frag(i, ag);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = aw_epi_mad(acc[i][j][e], ag[e], true, 0.f, false);
          ec_lds_w8(smem, nwb[i] + G::JS * j, ec_pack(v));
          ec_frag_fence(4 * j + i);
        }
      }
      ec_publish<G>(smem, L.w, L.lane, c + 1);
      ec_store_slice<G, WT>(smem, no, S, ec_rsrc(P.gh[r], nbytes));
    } else {
      // gx = gx' + (W1^T gh) * GELU'(x); go = gx * mask(block r - 1) (block r - 1's conv2 operand: the next operand
      // image) or, for r = 0, gx itself (the previous stage's weight-gradient operand, staged in the image)
      // raw (block 0): the scratch holds x_0, whose GELU' is evaluated here; otherwise the saved GELU'(x_r)
      auto grad = [&](int i, int j, float (&v)[4], auto raw) {
        float pv[4], gv[4], ag[4];
        pre_frag(i, pv);
        ec_unpack(gr[i][j], gv);
        if constexpr (decltype(raw)::value) {
          ec_gelu_grad4(pv, ag);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) ag[e] = pv[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = aw_epi_mad(acc[i][j][e], ag[e], true, gv[e], true);
        gr[i][j] = ec_pack(v);
      };
      if (r > 0) {
        const float dk = DROP ? 1.f / (1.f - P.drop_p) : 1.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          stage_pre(j);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v[4], ds[4] = {1.f, 1.f, 1.f, 1.f}, o[4];
            grad(i, j, v, std::false_type{});
            if constexpr (DROP) ec_scales(keep, i, j, dk, ds);
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = v[e] * ds[e];
            ec_lds_w8(smem, nwb[i] + G::JS * j, ec_pack(o));
            ec_frag_fence(4 * j + i);
          }
        }
        ec_publish<G>(smem, L.w, L.lane, c + 1);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          stage_pre(j);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v[4];
            grad(i, j, v, std::true_type{});
            ec_lds_w8(smem, nwb[i] + G::JS * j, gr[i][j]);
            ec_frag_fence(4 * j + i);
          }
        }
      }
      ec_store_slice<G, WT>(smem, no, S, ec_rsrc(P.gxo_out[r], nbytes));
    }
  }
}

// ---------------------------------------------------------------- fragment-packed weight copies
// Packed layout of a [512][K] matrix A (row m, k; K = 512 TAPS): the 1-KB block (m / 16, k / 32) at
// ((m / 16) * (K / 32) + k / 32) KB holds lane l = (m % 16) + 16 ((k % 32) / 8) at 16 l, element k % 8 within.
// Forward copies pack A = W ([out][(tap, in)]), backward copies A[i][(t, o)] = W[o][t * 512 + i] (per tap W_t^T).
struct PackJobs {
  const void* src[AW_RES_PACK_MAX];
  void* fwd[AW_RES_PACK_MAX];
  void* bwd[AW_RES_PACK_MAX];
};

// blockIdx = (x, job, kind), gridDim.x = 8 TAPS.  Both kinds stage through LDS so that the global reads and writes
// are whole lines (the first form, one 16-row block per workgroup with 16-B accesses at 256-B to 1-KB strides, took
// 28.7 us for the encoder step's 16 matrices).
//  kind 0: packed block rows mb = x, x + 8 TAPS, ..: W's rows 16 mb .. +15 (16 KB TAPS in and out): the packed block
//          row is a permutation of the 16 rows' 16-B chunks;
//  kind 1: tap t = x / 8, columns 64 b .. +63 (b = x % 8) of W_t (512 rows x 128 B) -> blocks (4b .. 4b + 3,
//          16 t .. 16 t + 15) of the backward copy.
constexpr int PK_PITCH1 = 128 + 16;       // kind 1 staging row pitch (conflict-free column reads)
template <int TAPS>
__global__ __launch_bounds__(256) void res_pack_kernel(PackJobs J) {
  constexpr int RB = EC_ROWB * TAPS, PITCH0 = RB + 16, KB = 16 * TAPS;   // source row bytes, kind 0 pitch, blocks/row
  constexpr int SZ = 16 * PITCH0 > EC_H * PK_PITCH1 ? 16 * PITCH0 : EC_H * PK_PITCH1;
  __shared__ __attribute__((aligned(16))) char t[SZ];
  const int x = blockIdx.x, job = blockIdx.y, tid = threadIdx.x;
  const char* __restrict__ W = reinterpret_cast<const char*>(J.src[job]);
  if (blockIdx.z == 0) {
    uint4* __restrict__ out = reinterpret_cast<uint4*>(J.fwd[job]);
    if (!out) return;
    for (int mb = x; mb < EC_H / 16; mb += gridDim.x) {
#pragma unroll
      for (int q = 0; q < 4 * TAPS; ++q) {   // 16 rows x 64 TAPS chunks, row-major: coalesced
        const int c = tid + 256 * q, row = c / (64 * TAPS), kc = c % (64 * TAPS);
        *reinterpret_cast<uint4*>(t + row * PITCH0 + kc * 16) =
            *reinterpret_cast<const uint4*>(W + (size_t)(16 * mb + row) * RB + kc * 16);
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 4 * TAPS; ++q) {   // output chunk o = (s, lane): row lane & 15, chunk 4s + (lane >> 4)
        const int o = tid + 256 * q, st = o >> 6, l = o & 63;
        out[(size_t)mb * 64 * KB + o] = *reinterpret_cast<const uint4*>(t + (l & 15) * PITCH0 + (4 * st + (l >> 4)) * 16);
      }
      __syncthreads();
    }
  } else {
    uint4* __restrict__ out = reinterpret_cast<uint4*>(J.bwd[job]);
    if (!out) return;
    const int tap = x >> 3, b = x & 7;
#pragma unroll
    for (int q = 0; q < 16; ++q) {    // W_t[o][64 b .. +63]: 512 rows x 8 chunks
      const int c = tid + 256 * q, o = c >> 3, kc = c & 7;
      *reinterpret_cast<uint4*>(t + o * PK_PITCH1 + kc * 16) =
          *reinterpret_cast<const uint4*>(W + (size_t)o * RB + tap * EC_ROWB + 128 * b + kc * 16);
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {    // 4 block rows x 16 blocks x 64 lanes, in output order
      const int o = tid + 256 * q, mb = o >> 10, st = (o >> 6) & 15, l = o & 63, li = l & 15, g = l >> 4;
      uint16_t e[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        e[k] = *reinterpret_cast<const uint16_t*>(t + (32 * st + 8 * g + k) * PK_PITCH1 + (16 * mb + li) * 2);
      uint4 v;
      memcpy(&v, e, 16);
      out[((size_t)(4 * b + mb) * KB + 16 * tap + st) * 64 + l] = v;
    }
  }
}

// Dropout keep bits of every chain lane (aw_res_dropout_masks): word ((r * nwg + wg) * 512 + tid) holds the 64 bits
// ec_scales reads, from the unfused epilogue's mask (aw_hash_group of block r's seed on group (row * H + c) >> 2) --
// what the forward chain computes in its K loops.
struct MaskSeeds {
  uint64_t seed[AW_RES_CHAIN_MAX];
};
__global__ __launch_bounds__(EC_NTH) void res_mask_kernel(MaskSeeds S, const uint64_t* seed_ptr, uint32_t thr,
                                                          u32x2* __restrict__ out) {
  const int tid = threadIdx.x, r = blockIdx.y;
  const int lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const uint64_t seed = aw_seed_mix(S.seed[r], seed_ptr);
  const uint64_t grp0 = (((uint64_t)blockIdx.x * EC_ROWS + li) * EC_H >> 2) + 16 * w + g;
  uint32_t k[2] = {0u, 0u};
#pragma unroll
  for (int f = 0; f < 16; ++f) k[f >> 3] |= ec_keep_bits(seed, grp0, f, thr);
  out[((size_t)r * gridDim.x + blockIdx.x) * EC_NTH + tid] = u32x2{k[0], k[1]};
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int TAPS>
void launch_fwd(const aw_res_chain_fwd_args* a, bool drop, bool wt, dim3 grid, hipStream_t s) {
  if (drop && wt) hipLaunchKernelGGL((res_chain_fwd_kernel<TAPS, true, true>), grid, dim3(EC_NTH), 0, s, *a);
  else if (drop) hipLaunchKernelGGL((res_chain_fwd_kernel<TAPS, true, false>), grid, dim3(EC_NTH), 0, s, *a);
  else if (wt) hipLaunchKernelGGL((res_chain_fwd_kernel<TAPS, false, true>), grid, dim3(EC_NTH), 0, s, *a);
  else hipLaunchKernelGGL((res_chain_fwd_kernel<TAPS, false, false>), grid, dim3(EC_NTH), 0, s, *a);
}
template <int TAPS>
void launch_bwd(const aw_res_chain_bwd_args* a, bool drop, bool wt, dim3 grid, hipStream_t s) {
  if (drop && wt) hipLaunchKernelGGL((res_chain_bwd_kernel<TAPS, true, true>), grid, dim3(EC_NTH), 0, s, *a);
  else if (drop) hipLaunchKernelGGL((res_chain_bwd_kernel<TAPS, true, false>), grid, dim3(EC_NTH), 0, s, *a);
  else if (wt) hipLaunchKernelGGL((res_chain_bwd_kernel<TAPS, false, true>), grid, dim3(EC_NTH), 0, s, *a);
  else hipLaunchKernelGGL((res_chain_bwd_kernel<TAPS, false, false>), grid, dim3(EC_NTH), 0, s, *a);
}

}  // namespace

#define CHAIN_SHAPE_CHECKS(who)                                                                                       \
  AW_REQUIRE(a, who ": null args");                                                                                   \
  AW_REQUIRE(a->H == EC_H, who ": H must be %d (got %d)", EC_H, a->H);                                                \
  AW_REQUIRE(a->R >= 1 && a->R <= AW_RES_CHAIN_MAX, who ": R must be 1..%d", AW_RES_CHAIN_MAX);                       \
  AW_REQUIRE(a->N >= 1 && (a->N + EC_ROWS) * EC_ROWB < (1ll << 31), who ": N out of range");                          \
  AW_REQUIRE(a->taps == 1 || (a->taps == 3 && a->seg == EC_SEG && a->N % EC_SEG == 0),                                \
             who ": taps must be 1, or 3 with seg == %d and N %% %d == 0 (taps %d, seg %d)", EC_SEG, EC_SEG, a->taps, \
             a->seg);                                                                                                 \
  AW_REQUIRE(a->drop_p >= 0.f && a->drop_p < 1.f, who ": drop_p out of [0, 1)")

extern "C" int aw_res_chain_fwd(const aw_res_chain_fwd_args* a, void* stream) {
  CHAIN_SHAPE_CHECKS("aw_res_chain_fwd");
  AW_REQUIRE(a->a0 && a->x0 && aligned16(a->a0) && aligned16(a->x0), "aw_res_chain_fwd: a0 / x0 missing or unaligned");
  for (int r = 0; r < a->R; ++r) {
    AW_REQUIRE(a->w1[r] && a->w2[r] && a->b1[r] && a->b2[r] && aligned16(a->w1[r]) && aligned16(a->w2[r]) &&
               aligned16(a->b1[r]) && aligned16(a->b2[r]), "aw_res_chain_fwd: block %d weights missing or unaligned", r);
    AW_REQUIRE(a->a[r] && aligned16(a->a[r]), "aw_res_chain_fwd: block %d output a missing or unaligned", r);
    AW_REQUIRE(aligned16(a->dgelu_h[r]) && aligned16(a->a1[r]) && aligned16(a->dgelu_x[r]),
               "aw_res_chain_fwd: block %d saved outputs unaligned", r);
  }
  AW_REQUIRE(aligned16(a->drop_masks), "aw_res_chain_fwd: drop_masks unaligned");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((a->N + EC_ROWS - 1) / EC_ROWS));
  const bool drop = a->drop_p > 0.f, wt = a->store_policy == AW_STORE_WT;
  if (a->taps == 3) launch_fwd<3>(a, drop, wt, grid, s);
  else launch_fwd<1>(a, drop, wt, grid, s);
  return aw::check_launch("aw_res_chain_fwd");
}

extern "C" int aw_res_chain_bwd(const aw_res_chain_bwd_args* a, void* stream) {
  CHAIN_SHAPE_CHECKS("aw_res_chain_bwd");
  AW_REQUIRE(a->gx && a->gxo && a->x0 && aligned16(a->gx) && aligned16(a->gxo) && aligned16(a->x0),
             "aw_res_chain_bwd: gx / gxo / x0 missing or unaligned");
  for (int r = 0; r < a->R; ++r) {
    AW_REQUIRE(a->w1t[r] && a->w2t[r] && aligned16(a->w1t[r]) && aligned16(a->w2t[r]),
               "aw_res_chain_bwd: block %d weights missing or unaligned", r);
    AW_REQUIRE(a->dgelu_h[r] && aligned16(a->dgelu_h[r]) && (r == 0 || (a->dgelu_x[r] && aligned16(a->dgelu_x[r]))),
               "aw_res_chain_bwd: block %d saved GELU' missing or unaligned", r);
    AW_REQUIRE(a->gh[r] && a->gxo_out[r] && aligned16(a->gh[r]) && aligned16(a->gxo_out[r]),
               "aw_res_chain_bwd: block %d outputs missing or unaligned", r);
  }
  AW_REQUIRE(a->drop_p == 0.f || a->R == 1 || (a->drop_masks && aligned16(a->drop_masks)),
             "aw_res_chain_bwd: drop_p > 0 needs drop_masks");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((a->N + EC_ROWS - 1) / EC_ROWS));
  const bool drop = a->drop_p > 0.f && a->R > 1, wt = a->store_policy == AW_STORE_WT;
  if (a->taps == 3) launch_bwd<3>(a, drop, wt, grid, s);
  else launch_bwd<1>(a, drop, wt, grid, s);
  return aw::check_launch("aw_res_chain_bwd");
}

extern "C" int aw_res_pack_weights(const void* const* src, void* const* fwd, void* const* bwd, int n, int taps,
                                   void* stream) {
  AW_REQUIRE(src && fwd && bwd && n >= 0 && n <= AW_RES_PACK_MAX && (taps == 1 || taps == 3),
             "aw_res_pack_weights: bad args (n must be 0..%d, taps 1 or 3)", AW_RES_PACK_MAX);
  if (n == 0) return AW_OK;
  PackJobs J{};
  for (int i = 0; i < n; ++i) {
    AW_REQUIRE(src[i] && aligned16(src[i]) && aligned16(fwd[i]) && aligned16(bwd[i]) && (fwd[i] || bwd[i]) &&
                   src[i] != fwd[i] && src[i] != bwd[i], "aw_res_pack_weights: job %d: missing, aliased or unaligned", i);
    J.src[i] = src[i];
    J.fwd[i] = fwd[i];
    J.bwd[i] = bwd[i];
  }
  const dim3 grid(8 * taps, n, 2);
  if (taps == 3) hipLaunchKernelGGL(res_pack_kernel<3>, grid, dim3(256), 0, (hipStream_t)stream, J);
  else hipLaunchKernelGGL(res_pack_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, J);
  return aw::check_launch("aw_res_pack_weights");
}

extern "C" int64_t aw_res_dropout_masks_bytes(int64_t N, int R) {
  if (N < 1 || R < 1 || R > AW_RES_CHAIN_MAX) return -1;
  return (int64_t)R * ((N + EC_ROWS - 1) / EC_ROWS) * EC_NTH * 8;
}

extern "C" int aw_res_dropout_masks(int64_t N, int R, float drop_p, const uint64_t* drop_seed, const uint64_t* seed_ptr,
                                    void* masks, void* stream) {
  AW_REQUIRE(N >= 1 && R >= 1 && R <= AW_RES_CHAIN_MAX && drop_seed && masks && aligned16(masks) && drop_p > 0.f &&
                 drop_p < 1.f, "aw_res_dropout_masks: bad args");
  MaskSeeds S{};
  for (int r = 0; r < R; ++r) S.seed[r] = drop_seed[r];
  hipLaunchKernelGGL(res_mask_kernel, dim3((unsigned)((N + EC_ROWS - 1) / EC_ROWS), R), dim3(EC_NTH), 0,
                     (hipStream_t)stream, S, seed_ptr, aw_drop_threshold(drop_p), (u32x2*)masks);
  return aw::check_launch("aw_res_dropout_masks");
}
