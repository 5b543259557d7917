// Weight gradients of the decoder's k = 3 / pad = 1 ResBlock convs (model/vq_vae_patch_embedd.py:60-74 via
// :142-145; the reference's autograd computes them through cuDNN's wgrad):
//   dW[o][j*I + i] += sum_t dy[t][o] * x[t + j - 1][i]   (x zero outside the token's window of `seg` tokens)
// as one launch over all (up to 16) convs of the ResBlock stack, bf16 operands, fp32 accumulation.
//
// gfx950 design (one workgroup per CU, 512 threads = 8 waves, 160 KB LDS):
//  * Tile = 256 output channels x (3 taps x 64 input channels).  Both operands are token-major ([K][rows]), so each
//    K-tile of 64 tokens stages dy[64][256] (32 KB) and ONE x[64][64] image (8 KB) that serves all three taps: tap j
//    reads the x rows shifted by j - 1 (the shift never leaves a window, and windows never straddle a 64-token
//    K-tile since seg | 64).  The taps' window masks are one AND per B fragment (element 0 for j = 0, element 7
//    for j = 2, on the lanes whose token sits at a window edge).  Decoder shape (16 convs, O = I = 512):
//    2 x 8 tiles per conv = 256 tiles = one per CU, every tile owns its output block -> no split-K, no atomics:
//    the epilogue adds into the gradient with plain read-modify-write.
//  * Four LDS buffers of 40 KB: LDS-DMA (buffer_load ... lds) of K-tile t + 3 is issued inside the MFMA segment of
//    tile t (hidden among the MFMAs), each wave retires its own DMA with a counted vmcnt (never 0 in the loop) two
//    tiles later and a barrier publishes it.
//  * Two wave groups ping-pong (the guide's 8-wave schedule): group 1 runs one barrier behind group 0, so while one
//    group issues its 44 ds_read_b64_tr_b16 (one lane base per operand, immediate offsets) the other runs its 48
//    MFMAs (v_mfma_f32_16x16x32_bf16, 128 x 48 outputs per wave); the reads are waited for at their first use.
//  * LDS images are [16-row block][64 k][16 rows] with the k field XOR-swizzled (k ^ (bit3(k) << 2)): every
//    transposed read of a 32-lane half hits 8 distinct 32-B slots (conflict-free for all three tap shifts), and the
//    A-fragment addresses are one lane base + immediate offsets.  The swizzle is applied to the DMA source address
//    (the image is lane-linear per DMA instruction).
#include "gemm_core.h"

#include <stdlib.h>

#include <algorithm>

#pragma clang diagnostic ignored "-Winline-asm"

namespace {

constexpr int W3_BM = 256;                 // output rows (o) per tile
constexpr int W3_CB = 64;                  // input channels per tile (x 3 taps = 192 output columns)
constexpr int W3_BK = 64;                  // tokens per K-tile
constexpr int W3_NTH = 512;
constexpr int W3_A = W3_BK * W3_BM * 2;    // 32768 B: dy image
constexpr int W3_B = W3_BK * W3_CB * 2;    // 8192 B: x image
constexpr int W3_BUF = W3_A + W3_B;        // 40960 B
constexpr int W3_NBUF = 4;                 // 163840 B = the whole LDS of a CU
constexpr int W3_DMA = 5;                  // DMA instructions per thread per K-tile (4 dy + 1 x)
// The DMA of K-tile t + 3 is issued in the read segment of tile t (which then retires its reads before the barrier):
// measured faster than issuing it inside the MFMA segment, or t + 2 in the read segment (round-3 probes).

struct W3Params {
  int M, cin, K, seg, ngroups, tiles_m, tiles_i, nblocks;
  int lda, ldb, ldc;
  int col_mod, col_mul, col_off;
  float alpha;
  const void* A[AW_GEMM_MAX_GROUPS];       // dy [K][lda] bf16
  const void* B[AW_GEMM_MAX_GROUPS];       // x  [K][ldb] bf16
  float* C[AW_GEMM_MAX_GROUPS];            // dW [M][ldc] f32 (columns through the col map)
  float* rowsum[AW_GEMM_MAX_GROUPS];       // bias gradient (NULL: none)
};

typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// byte of the swizzled k field: the k row lives at 32 * (k ^ (bit3(k) << 2)) inside its 16-row block
__device__ __forceinline__ int w3_kfield(int k) { return 32 * (k ^ (((k >> 3) & 1) << 2)); }

__device__ __forceinline__ v4i32 w3_desc(const void* base) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  return v4i32{(int)__builtin_amdgcn_readfirstlane((uint32_t)b),
               (int)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu), 0x7FFFFFFF, 0x00020000};
}

__device__ __forceinline__ void w3_dma(uint32_t m0, int off, v4i32 desc) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(desc)
               : "memory", "m0");
}

__device__ __forceinline__ uint4 w3_tr(const char* p_lo, const char* p_hi) {
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(uintptr_t)p_lo);
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(uintptr_t)p_hi);
  uint4 out;
  memcpy(&out, &lo, 8);
  memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
  return out;
}

template <int N> __device__ __forceinline__ void w3_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ void w3_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}


__global__ __launch_bounds__(W3_NTH, 1) void wgrad_conv3_kernel(W3Params P) {
  __shared__ __attribute__((aligned(16))) char smem[W3_NBUF * W3_BUF];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;           // wave group (M half) and N quarter
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;

  int unit = awg::xcd_remap(blockIdx.x, P.nblocks);
  const int per_group = P.tiles_m * P.tiles_i;
  const int grp = unit / per_group;
  unit -= grp * per_group;
  const int tm = unit / P.tiles_i, ti = unit % P.tiles_i;
  const int m0 = tm * W3_BM, ci0 = ti * W3_CB;
  const char* Ag = reinterpret_cast<const char*>(P.A[grp]) + (int64_t)m0 * 2;
  const char* Bg = reinterpret_cast<const char*>(P.B[grp]) + (int64_t)ci0 * 2;

  // ---- DMA source offsets (bytes, K-tile 0) of this thread's chunks; the image is lane-linear: chunk c of a
  //      K-tile lands at byte 16 c of the image
  int offA[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + W3_NTH * i;
    const int mb = c >> 7, w = c & 127;
    const int kf = w >> 1, half = w & 1;
    const int k = kf ^ (((kf >> 3) & 1) << 2);
    offA[i] = (k * P.lda + mb * 16 + half * 8) * 2;
  }
  int offB;
  {
    const int c = tid;
    const int cb = c >> 7, w = c & 127;
    const int kf = w >> 1, half = w & 1;
    const int k = kf ^ (((kf >> 3) & 1) << 2);
    offB = (k * P.ldb + cb * 16 + half * 8) * 2;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const uint32_t wave_dst = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tid & ~63)) * 16u;
  const int64_t a_step = (int64_t)W3_BK * P.lda * 2, b_step = (int64_t)W3_BK * P.ldb * 2;

  auto dma = [&](int t) {
    const uint32_t buf = lds0 + (uint32_t)((t & (W3_NBUF - 1)) * W3_BUF);
    const v4i32 da = w3_desc(Ag + t * a_step);
    const v4i32 db = w3_desc(Bg + t * b_step);
#pragma unroll
    for (int i = 0; i < 4; ++i) w3_dma(buf + wave_dst + (uint32_t)(i * W3_NTH * 16), offA[i], da);
    w3_dma(buf + W3_A + wave_dst, offB, db);
  };

  // ---- fragment addresses (bytes within a buffer)
  // A fragment (i, u, h): block mb = wr*8 + i, k = 32u + 8g + 4h + q, rows 4p..4p+3 of the block
  const int a_lo = w3_kfield(8 * g + q) + 8 * p;           // h = 0  (+ 1024 u + 2048 mb, no carry: see kfield)
  const int a_hi = w3_kfield(8 * g + 4 + q) + 8 * p;       // h = 1
  // B fragment f of this wave: output column c = wc*48 + 16 f -> tap j = c / 64, channel block cb = (c % 64) / 16;
  // rows shifted by j - 1 (wrapped into the image: only masked elements read a wrapped row)
  // u = 1 adds 32 rows = 1024 bytes to the swizzled address for every row r < 32 (kfield leaves bit 5 alone); the
  // rows that leave the image (r = -1 or 64: tap 0 / tap 2 at a window edge) only feed masked elements, and their
  // addresses stay inside this buffer
  int b_base[3][2];
  int tap[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int c = wc * 48 + 16 * f;
    const int j = c >> 6, cb = (c & 63) >> 4;
    tap[f] = j;
#pragma unroll
    for (int h = 0; h < 2; ++h) b_base[f][h] = W3_A + cb * 2048 + w3_kfield((8 * g + 4 * h + q + j - 1) & 63) + 8 * p;
  }
  // window masks: element 0 of the fragment (token 32u + 8g) for tap 0, element 7 (token 32u + 8g + 7) for tap 2;
  // branch-free per fragment (all-ones for the other taps)
  const uint32_t mask_e0 = ((8 * g) % P.seg == 0) ? 0xFFFF0000u : 0xFFFFFFFFu;
  const uint32_t mask_e7 = ((8 * g + 8) % P.seg == 0) ? 0x0000FFFFu : 0xFFFFFFFFu;
  uint32_t mlo[3], mhi[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    mlo[f] = tap[f] == 0 ? mask_e0 : 0xFFFFFFFFu;
    mhi[f] = tap[f] == 2 ? mask_e7 : 0xFFFFFFFFu;
  }

  float* rowptr = P.rowsum[grp];
  // bias gradient (row sums of dy over the tokens): every tile of a row block takes every tiles_i-th K-tile, and within a
  // tile the group's 4 waves share the work: wave wc sums A fragments 2wc and 2wc + 1 with an MFMA against an all-ones
  // B fragment (4 extra MFMAs on those K-tiles; a VALU sum of all 16 fragments in one wave of the ti == 0 tiles
  // cost ~1000 cycles per K-tile on the critical path)
  const bool tile_rowsum = rowptr != nullptr;
  int rs_count = ti;        // this tile sums K-tiles t == ti (mod tiles_i): the work is spread over the row's tiles
  const int wcu = __builtin_amdgcn_readfirstlane(wc);
  const uint4 ones = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  f32x4 rs[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

  f32x4 acc[8][3];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int f = 0; f < 3; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = P.K / W3_BK;
  // ---- prologue: K-tiles 0..2 in flight, tile 0 retired and published
  dma(0);
  if (nk > 1) dma(1);
  if (nk > 2) dma(2);
  if (nk > 2) w3_vmcnt<2 * W3_DMA>();
  else if (nk > 1) w3_vmcnt<W3_DMA>();
  else w3_vmcnt<0>();
  w3_barrier();
  if (wr == 1) w3_barrier();                         // group 1 runs one barrier behind group 0

  uint4 af[2][8], bfr[2][3];
  for (int t = 0; t < nk; ++t) {
    // ---- read segment: this group's fragments of K-tile t, the DMA of t + 3, retire t + 1
    const char* buf = smem + (t & (W3_NBUF - 1)) * W3_BUF;
    {
      // one lane base per read kind, the rest as immediate offsets of the ds_read instructions
      const char* pa_lo = buf + wr * 8 * 2048 + a_lo;
      const char* pa_hi = buf + wr * 8 * 2048 + a_hi;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 8; ++i) af[u][i] = w3_tr(pa_lo + (i * 2048 + 1024 * u), pa_hi + (i * 2048 + 1024 * u));
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const char* pb_lo = buf + b_base[f][0];
        const char* pb_hi = buf + b_base[f][1];
#pragma unroll
        for (int u = 0; u < 2; ++u) bfr[u][f] = w3_tr(pb_lo + 1024 * u, pb_hi + 1024 * u);
      }
    }
    // DMA of K-tile t + 3 into buffer (t - 1) % 4: the other group read tile t - 1 in the previous segment and retired
    // those reads before the barrier (the lgkmcnt(0) below), so the buffer is free
    if (t + 3 < nk) dma(t + 3);
    const int newer = min(nk - 1, t + 3) - (t + 1);   // tiles issued after t + 1 (still allowed in flight)
    if (newer >= 2) w3_vmcnt<2 * W3_DMA>();
    else if (newer == 1) w3_vmcnt<W3_DMA>();
    else w3_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this buffer's reads retire before the barrier (WAR)
    // the window masks while the reads are retired anyway: the MFMA segment opens with MFMAs (no VALU head)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        bfr[u][f].x &= mlo[f];
        bfr[u][f].w &= mhi[f];
      }
    // otherwise the reads' own lgkmcnt waits come at their first use in the MFMA segment: their latency overlaps the
    // barrier and the other group's MFMAs
    w3_barrier();
    // ---- MFMA segment
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int f = 0; f < 3; ++f)
          acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[u][i]),
                                                             __builtin_bit_cast(bf16x8, bfr[u][f]), acc[i][f], 0, 0, 0);
    }
    const bool rs_now = tile_rowsum && rs_count == 0;
    rs_count = rs_count == 0 ? P.tiles_i - 1 : rs_count - 1;
    if (rs_now) {
#define W3_RS(a, b)                                                                                                \
  for (int u = 0; u < 2; ++u) {                                                                                   \
    rs[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[u][a]),                          \
                                                    __builtin_bit_cast(bf16x8, ones), rs[0], 0, 0, 0);             \
    rs[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[u][b]),                          \
                                                    __builtin_bit_cast(bf16x8, ones), rs[1], 0, 0, 0);             \
  }
      switch (wcu) {            // wave-uniform: static fragment indices (no dynamic register indexing)
        case 0: W3_RS(0, 1) break;
        case 1: W3_RS(2, 3) break;
        case 2: W3_RS(4, 5) break;
        default: W3_RS(6, 7) break;
      }
#undef W3_RS
    }
    __builtin_amdgcn_s_setprio(0);
    w3_barrier();
  }
  if (wr == 0) w3_barrier();                         // both groups end on the same barrier count

  // ---- epilogue: this tile owns its output block -> plain read-modify-write of the f32 gradient
  const float alpha = P.alpha;
  float* C = P.C[grp];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int c = wc * 48 + 16 * f + li;
    const int n = (c >> 6) * P.cin + ci0 + (c & 63);
    const int64_t oc = P.col_mod > 0 ? (int64_t)(n % P.col_mod) * P.col_mul + n / P.col_mod + P.col_off
                                     : (int64_t)n * (P.col_mul > 0 ? P.col_mul : 1) + P.col_off;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = m0 + wr * 128 + 16 * i + 4 * g;
      float* d = C + (int64_t)row * P.ldc + oc;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = d[(int64_t)r * P.ldc];
#pragma unroll
      for (int r = 0; r < 4; ++r) d[(int64_t)r * P.ldc] = v[r] + alpha * acc[i][f][r];
    }
  }
  if (tile_rowsum && li == 0) {   // column 0 of D = A . ones: lane 16g holds rows 4g..4g+3 of the fragment
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(rowptr + m0 + wr * 128 + 16 * (2 * wcu + j) + 4 * g + r, alpha * rs[j][r]);
  }
}

int g_policy = 0;   // aw_gemm_set_wgrad_policy: 0 automatic, 1 force, -1 off

// =====================================================================================================================
// Weight gradients of plain (1-tap) layers, a batch of problems of any (M, N) sharing K in ONE stream-K launch:
//   dW_p[m][colmap(n)] += alpha * sum_k A_p[k][m] * B_p[k][n]      (A = dy [K][lda], B = x [K][ldb], bf16, f32 acc)
//   rowsum_p[m]        += alpha * sum_k A_p[k][m]                  (bias gradient)
// The transformer's four Linear kinds of half the blocks (model/transformer_block.py:28-30,76-77 grads, K = the B*T
// tokens, ragged) and the VQ-VAE encoder's 16 centre-tap convs (model/vq_vae_patch_embedd.py:65,68 via :108-110).
//  * Tile 256 x 256, K-stage 32 tokens, 512 threads in two wave groups that ping-pong (wgrad_conv3_kernel's schedule):
//    each wave owns 128 x 64 outputs (8 x 4 fragments of v_mfma_f32_16x16x32_bf16); per stage a wave reads 12
//    transposed fragments (24 ds_read_b64_tr_b16) and issues 32 MFMAs.  Four 32 KB stages (128 KB of LDS) filled by
//    LDS-DMA three stages ahead; the tails of a ragged K read zeros from the buffer range check.
//  * Split-K with k-ALIGNED units: tile t is cut into S equal token ranges (S = 4 at the bench shapes: the
//    transformer's 192 tiles -> 768 units = three full rounds of 256 CUs, the encoder's 64 -> one round); persistent
//    workgroups (one per CU) take units u = c, c + G, ... in split-major order, so the workgroups that run together
//    are at the same k of their ranges, and the tiles that share an operand block sit on one XCD: their operand
//    streams meet in that XCD's L2.  (A stream-K cut into equal contiguous ranges, measured first, put concurrent
//    workgroups at different k: 3.2 GB fetched per transformer half-step, slower than the per-kind launches.)
//  * A tile's S partial pieces are summed by the LAST arriving piece: each piece takes an arrival ticket (one agent-
//    scope atomic add) when its loop ends; every piece but the last stores its accumulators write-through (sc1) into
//    its workspace slot, drains them (vmcnt(0)), joins a workgroup barrier and counts itself published (one more
//    atomic add); the last polls the published count with sc1 loads (a poll that never completes traps instead of
//    summing unwritten slots), then loads the other slots with sc1 loads and
//    does the one read-modify-write of the gradient (MI355X_MICROARCH.md, inter-workgroup hand-off, first row of the
//    measured forms).  It waits only for pieces that already hold tickets, i.e. are running and only store: no
//    deadlock whatever the residency.  The read-modify-write goes through LDS in two 128-row halves: float4 per lane, 16 row loads in flight.
//  * Bias gradients: row sums of the A fragments by MFMA against an all-ones fragment, on the stages s with
//    s % tiles_n == tn (spread over the row's tiles), f32 atomics per piece.
constexpr int WT_BM = 256, WT_BN = 256, WT_BK = 32, WT_NTH = 512;
constexpr int WT_A = WT_BK * WT_BM * 2;      // 16384 B
constexpr int WT_B = WT_BK * WT_BN * 2;      // 16384 B
constexpr int WT_BUF = WT_A + WT_B;          // 32768 B
constexpr int WT_NBUF = 4;                   // 131072 B
constexpr int WT_DMA = 4;                    // DMA instructions per thread per stage (2 A + 2 B)
constexpr int WT_SLAB = WT_BM * WT_BN;       // f32 elements of one partial tile
constexpr int WT_MAXTILES = 8192;

struct WTProb {
  const void* A;
  const void* B;
  float* C;
  float* rowsum;
  int64_t lda, ldb, ldc;
  int M, N, tiles_n, tile0;
  int col_mod, col_mul, col_off;
};

struct WTParams {
  WTProb p[AW_WGRAD_BATCH_MAX];   // 32 x 88 B: the kernel-argument block stays under 3 KB
  int nprob, K, nk, G, total_tiles, S, units;
  int big;            // tiles [0, big) run unsplit (one full-K unit each), the rest in S k-aligned pieces
  float alpha;
  float* ws;          // one slot of WT_SLAB floats per unit
  int spin;           // poll bound of the fix-up (aw_wgrad_set_spin_limit; 0 forces the broken-hand-off path)
};

// per-tile counters of arrived and of published pieces; the last arriver resets both of its tile to 0
__device__ int g_wt_arrive[WT_MAXTILES];
__device__ int g_wt_pub[WT_MAXTILES];

__device__ __forceinline__ v4i32 wt_desc(const void* base, int64_t nbytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const int64_t nb = nbytes < 0 ? 0 : (nbytes > 0x7FFFFFF0 ? 0x7FFFFFF0 : nbytes);
  return v4i32{(int)__builtin_amdgcn_readfirstlane((uint32_t)b),
               (int)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu),
               (int)__builtin_amdgcn_readfirstlane((uint32_t)nb), 0x00020000};
}


__device__ __forceinline__ void wt_st_sc1(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__global__ __launch_bounds__(WT_NTH, 1) void wgrad_tt_kernel(WTParams P) {
  __shared__ __attribute__((aligned(16))) char smem[WT_NBUF * WT_BUF];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
  const int wcu = __builtin_amdgcn_readfirstlane(wc);
  const int c = awg::xcd_remap(blockIdx.x, P.G);      // logical workgroup: consecutive ranges share an XCD's L2
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const uint32_t wave_dst = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tid & ~63)) * 16u;
  const uint4 ones = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  // fragment addresses within a stage buffer: A block mb = wr*8 + i at mb*1024, B block cb = wc*4 + f at WT_A + cb*1024
  const int f_lo = w3_kfield(8 * g + q) + 8 * p4, f_hi = w3_kfield(8 * g + 4 + q) + 8 * p4;
  // DMA chunk c = tid + 512 j of an image: block mb = c >> 6, k field kf = (c & 63) >> 1, half = c & 1
  int src_row[2], src_col[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ch = tid + WT_NTH * j;
    const int kf = (ch & 63) >> 1;
    src_row[j] = kf ^ (((kf >> 3) & 1) << 2);
    src_col[j] = (ch >> 6) * 16 + (ch & 1) * 8;
  }

  for (int unit = c; unit < P.units; unit += P.G) {
    // units [0, big): tile = unit, full K; then the split tiles' pieces, split-major: piece sp of split tile t is unit
    // big + sp * nsplit + (t - big) = sp * nsplit + t (big = 0: the uniform plan)
    const int nsplit = P.total_tiles - P.big;
    int tile, sp, St;
    if (unit < P.big) {
      tile = unit, sp = 0, St = 1;
    } else {
      sp = (unit - P.big) / nsplit;
      tile = unit - sp * nsplit;
      St = P.S;
    }
    const int k0 = (int)((int64_t)sp * P.nk / St), k1 = (int)((int64_t)(sp + 1) * P.nk / St);
    int pi = 0;
    while (pi + 1 < P.nprob && tile >= P.p[pi + 1].tile0) ++pi;
    const WTProb& pr = P.p[pi];
    const int lt = tile - pr.tile0;
    const int tm = lt / pr.tiles_n, tn = lt - tm * pr.tiles_n;
    const int m0 = tm * WT_BM, n0 = tn * WT_BN;
    const char* Ag = reinterpret_cast<const char*>(pr.A) + (int64_t)m0 * 2;
    const char* Bg = reinterpret_cast<const char*>(pr.B) + (int64_t)n0 * 2;
    const int64_t lda = pr.lda, ldb = pr.ldb;
    int offA[2], offB[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      offA[j] = (int)((src_row[j] * lda + src_col[j]) * 2);
      offB[j] = (int)((src_row[j] * ldb + src_col[j]) * 2);
    }
    const int64_t extA = ((int64_t)(P.K - 1) * lda + pr.M - m0) * 2;   // valid bytes from the tile's row 0
    const int64_t extB = ((int64_t)(P.K - 1) * ldb + pr.N - n0) * 2;
    auto dma = [&](int t) {
      const uint32_t buf = lds0 + (uint32_t)((t & (WT_NBUF - 1)) * WT_BUF);
      const int64_t ra = (int64_t)t * WT_BK * lda * 2, rb = (int64_t)t * WT_BK * ldb * 2;
      const v4i32 da = wt_desc(Ag + ra, extA - ra), db = wt_desc(Bg + rb, extB - rb);
#pragma unroll
      for (int j = 0; j < 2; ++j) w3_dma(buf + wave_dst + (uint32_t)(j * WT_NTH * 16), offA[j], da);
#pragma unroll
      for (int j = 0; j < 2; ++j) w3_dma(buf + WT_A + wave_dst + (uint32_t)(j * WT_NTH * 16), offB[j], db);
    };
    float* rowptr = pr.rowsum;
    f32x4 rs[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- prologue: stages k0 .. k0+2 in flight, k0 retired and published
    const int ns = k1 - k0;
    dma(k0);
    if (ns > 1) dma(k0 + 1);
    if (ns > 2) dma(k0 + 2);
    if (ns > 2) w3_vmcnt<2 * WT_DMA>();
    else if (ns > 1) w3_vmcnt<WT_DMA>();
    else w3_vmcnt<0>();
    w3_barrier();
    if (wr == 1) w3_barrier();                 // group 1 runs one barrier behind group 0

    uint4 af[8], bfr[4];
    for (int t = k0; t < k1; ++t) {
      // ---- read segment: fragments of stage t, the DMA of t + 3 (into the buffer of t - 1, read by both groups
      //      before the last barrier), retire t + 1
      const char* buf = smem + (t & (WT_NBUF - 1)) * WT_BUF;
      {
        const char* pa_lo = buf + wr * 8 * 1024 + f_lo;
        const char* pa_hi = buf + wr * 8 * 1024 + f_hi;
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = w3_tr(pa_lo + i * 1024, pa_hi + i * 1024);
        const char* pb_lo = buf + WT_A + wc * 4 * 1024 + f_lo;
        const char* pb_hi = buf + WT_A + wc * 4 * 1024 + f_hi;
#pragma unroll
        for (int f = 0; f < 4; ++f) bfr[f] = w3_tr(pb_lo + f * 1024, pb_hi + f * 1024);
      }
      if (t + 3 < k1) dma(t + 3);
      const int newer = min(k1 - 1, t + 3) - (t + 1);
      if (newer >= 2) w3_vmcnt<2 * WT_DMA>();
      else if (newer == 1) w3_vmcnt<WT_DMA>();
      else w3_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      w3_barrier();
      // ---- MFMA segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int f = 0; f < 4; ++f)
          acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                             __builtin_bit_cast(bf16x8, bfr[f]), acc[i][f], 0, 0, 0);
      if (rowptr != nullptr && t % pr.tiles_n == tn) {
#define WT_RS(a, b)                                                                                              \
  rs[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[a]), __builtin_bit_cast(bf16x8, ones), \
                                                  rs[0], 0, 0, 0);                                                \
  rs[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[b]), __builtin_bit_cast(bf16x8, ones), \
                                                  rs[1], 0, 0, 0);
        switch (wcu) {
          case 0: WT_RS(0, 1) break;
          case 1: WT_RS(2, 3) break;
          case 2: WT_RS(4, 5) break;
          default: WT_RS(6, 7) break;
        }
#undef WT_RS
      }
      __builtin_amdgcn_s_setprio(0);
      w3_barrier();
    }
    if (wr == 0) w3_barrier();                 // both groups end on the same barrier count

    const float alpha = P.alpha;
    if (rowptr != nullptr && li == 0) {         // column 0 of A . ones: lane 16g holds rows 4g..4g+3
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = rs[j][r];
          if (v != 0.f) atomicAdd(rowptr + m0 + wr * 128 + 16 * (2 * wcu + j) + 4 * g + r, alpha * v);
        }
    }
    bool write = true;
    if (St > 1) {
      // ---- one piece of S: take an arrival ticket first; the last to arrive sums the other pieces once they have
      //      published (they took their tickets before it, so they are resident and only store, drain and count: the
      //      wait is bounded whatever the residency), the others publish their accumulators and leave
      if (tid == 0) s_last = __hip_atomic_fetch_add(&g_wt_arrive[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                             St - 1;
      __syncthreads();
      write = s_last != 0;
      if (!write) {
        float* mine = P.ws + (int64_t)unit * WT_SLAB;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int f = 0; f < 4; ++f) wt_st_sc1(mine + ((i * 4 + f) * WT_NTH + tid) * 4, acc[i][f]);
        // the sc1 hand-off form of MI355X_MICROARCH.md (valid forms, first table row): every storing wave drains its
        // write-through stores, a workgroup barrier, then ONE lane's agent-scope add.  Not the memory model's
        // release / acquire fences: their L2 write-back (buffer_wbl2) and invalidates cost the decoder step
        // 5.34 -> 6.29 ms (same-box A/B, four alternating runs)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(&g_wt_pub[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        if (tid == 0) {
          // poll of the published count: a bounded spin (the publishers took their tickets first, so they are
          // resident and only store, drain and count); running out of it means a broken hand-off, which must not
          // turn into a silently wrong gradient: trap
          int it = 0;   // relaxed agent loads = sc1 loads: past this CU's L1
          for (; it < P.spin; ++it) {
            if (__hip_atomic_load(&g_wt_pub[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= St - 1) break;
            __builtin_amdgcn_s_sleep(1);
          }
          // a broken hand-off poisons the tile (NaN: loud in the loss, the clip norm and every check) instead of
          // summing unwritten slots silently
          if (it == P.spin) acc[0][0] = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), 0.f};
          __hip_atomic_store(&g_wt_pub[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&g_wt_arrive[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();   // the polling wave joins: every wave's slot loads (all sc1) come after the poll matched
        for (int o = 0; o < St; ++o) {
          if (o == sp) continue;
          const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(P.ws + ((int64_t)o * nsplit + tile) * WT_SLAB,
                                                              (short)0, WT_SLAB * 4, 0x00020000);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int f = 0; f < 4; ++f) {
              // sc1 load (cache policy bit 4): served past this CU's L1, as the hand-off requires
              const f32x4 v = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((i * 4 + f) * WT_NTH + tid) * 16, 0, 16));
              acc[i][f] += v;
            }
        }
      }
    }
    if (write) {
      // ---- the tile's one read-modify-write of the gradient, through LDS in two 128-row halves (the stage ring is
      //      free: every wave passed the loop's last barrier): lane-contiguous float4 columns, 16 rows in flight
      float* C = pr.C;
      float* T = reinterpret_cast<float*>(smem);                // [128][WT_BN] f32 = 128 KB
      const bool vec = pr.col_mod == 0 && pr.col_mul <= 1 && (pr.ldc & 3) == 0 && (pr.col_off & 3) == 0 &&
                       (((uintptr_t)C) & 15) == 0;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if (hh) __syncthreads();                                 // the first half's reads are done
        if (wr == hh) {
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
              for (int r = 0; r < 4; ++r) T[(16 * i + 4 * g + r) * WT_BN + wc * 64 + 16 * f + li] = acc[i][f][r];
        }
        __syncthreads();
        const int row0 = m0 + 128 * hh;
        if (vec) {
          const int c4 = (tid & 63) * 4, rr = tid >> 6;           // 64 float4 per row, 8 rows per pass
#pragma unroll
          for (int k0r = 0; k0r < 16; k0r += 8) {                 // 8 rows of loads in flight per lane
            f32x4 old[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
              old[k] = *reinterpret_cast<const f32x4*>(C + (int64_t)(row0 + rr + 8 * (k0r + k)) * pr.ldc + pr.col_off +
                                                       n0 + c4);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const f32x4 a = *reinterpret_cast<const f32x4*>(T + (rr + 8 * (k0r + k)) * WT_BN + c4);
              *reinterpret_cast<f32x4*>(C + (int64_t)(row0 + rr + 8 * (k0r + k)) * pr.ldc + pr.col_off + n0 + c4) =
                  old[k] + alpha * a;
            }
          }
        } else {
          const int cc = tid & 255, rr = tid >> 8;                // one column per lane, 2 rows per pass
          const int n = n0 + cc;
          const int64_t oc = pr.col_mod > 0 ? (int64_t)(n % pr.col_mod) * pr.col_mul + n / pr.col_mod + pr.col_off
                                            : (int64_t)n * (pr.col_mul > 0 ? pr.col_mul : 1) + pr.col_off;
          for (int k = 0; k < 64; k += 8) {
            float old[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) old[e] = C[(int64_t)(row0 + rr + 2 * (k + e)) * pr.ldc + oc];
#pragma unroll
            for (int e = 0; e < 8; ++e)
              C[(int64_t)(row0 + rr + 2 * (k + e)) * pr.ldc + oc] = old[e] + alpha * T[(rr + 2 * (k + e)) * WT_BN + cc];
          }
        }
      }
    }
    __syncthreads();     // the epilogue's LDS reads are done before the next unit's DMA refills the ring
  }
}

// ---- host side of the batch
int g_cus = 0;
int g_wt_spin = 1 << 26;   // the fix-up's poll bound (aw_wgrad_set_spin_limit)

int wt_cus() {
  if (g_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && n > 0)
      g_cus = n;
    else
      g_cus = 256;
  }
  return g_cus;
}

// checks + launch plan; P == nullptr: only validate.  Returns AW_OK, or a negative status (with the message set)
int wt_plan(const aw_gemm_args* args, int n, WTParams* P) {
  AW_REQUIRE(args && n >= 1 && n <= AW_WGRAD_BATCH_MAX, "aw_wgrad_batch: need 1..%d problems", AW_WGRAD_BATCH_MAX);
  const aw_gemm_args& a0 = args[0];
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const aw_gemm_args& a = args[i];
    AW_REQUIRE(a.a_dtype == AW_BF16 && a.a_trans == 1 && a.b_trans == 1 && a.conv_cin == 0,
               "aw_wgrad_batch: problem %d: bf16 operands, a_trans = b_trans = 1, no conv", i);
    AW_REQUIRE(a.accumulate == 1 && a.c_dtype == AW_F32 && a.C && a.beta == 0.f && !a.bias && !a.pre && !a.resid &&
                   !a.C2 && !a.colstats && a.drop_p <= 0.f,
               "aw_wgrad_batch: problem %d: accumulate-mode f32 C only", i);
    AW_REQUIRE(a.K == a0.K && a.alpha == a0.alpha, "aw_wgrad_batch: problem %d: K and alpha must match problem 0", i);
    AW_REQUIRE(a.M > 0 && a.N > 0 && a.M % WT_BM == 0 && a.N % WT_BN == 0,
               "aw_wgrad_batch: problem %d: M, N must be positive multiples of 256 (got %d x %d)", i, a.M, a.N);
    AW_REQUIRE(a.A && a.B && ((uintptr_t)a.A % 16) == 0 && ((uintptr_t)a.B % 16) == 0 && a.lda % 8 == 0 &&
                   a.ldb % 8 == 0 && a.lda >= a.M && a.ldb >= a.N,
               "aw_wgrad_batch: problem %d: 16-B aligned operand rows with lda >= M, ldb >= N", i);
    AW_REQUIRE((int64_t)WT_BK * a.lda * 2 < 0x7FFFFFF0 && (int64_t)WT_BK * a.ldb * 2 < 0x7FFFFFF0,
               "aw_wgrad_batch: problem %d: leading dimension too large", i);
    tiles += (a.M / WT_BM) * (a.N / WT_BN);
  }
  AW_REQUIRE(a0.K > 0, "aw_wgrad_batch: K must be positive");
  // each tile read-modify-writes its block of C once, without atomics: problems must not share C storage (the
  // extent of problem i's rows: [C, C + M * ldc) floats)
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const uintptr_t bi = (uintptr_t)args[i].C, ei = bi + (uintptr_t)args[i].M * args[i].ldc * sizeof(float);
      const uintptr_t bj = (uintptr_t)args[j].C, ej = bj + (uintptr_t)args[j].M * args[j].ldc * sizeof(float);
      AW_REQUIRE(ei <= bj || ej <= bi, "aw_wgrad_batch: problems %d and %d write overlapping C storage", i, j);
    }
  AW_REQUIRE(tiles <= WT_MAXTILES, "aw_wgrad_batch: %d tiles exceed %d", tiles, WT_MAXTILES);
  if (!P) return AW_OK;
  memset(P, 0, sizeof(*P));
  int t0 = 0;
  for (int i = 0; i < n; ++i) {
    const aw_gemm_args& a = args[i];
    WTProb& q = P->p[i];
    q.A = a.A;
    q.B = a.B;
    q.C = reinterpret_cast<float*>(a.C);
    q.rowsum = a.a_rowsum;
    q.lda = a.lda;
    q.ldb = a.ldb;
    q.ldc = a.ldc;
    q.M = a.M;
    q.N = a.N;
    q.tiles_n = a.N / WT_BN;
    q.tile0 = t0;
    q.col_mod = a.col_mod;
    q.col_mul = a.col_mul;
    q.col_off = a.col_off;
    t0 += (a.M / WT_BM) * q.tiles_n;
  }
  P->nprob = n;
  P->K = a0.K;
  P->nk = (a0.K + WT_BK - 1) / WT_BK;
  P->total_tiles = tiles;
  // split count: the fewest stages per CU over whole rounds of units, S <= 4 (the last arriver then reads at most
  // three partial tiles) and >= 16 stages per unit; ties go to the smaller S
  const int cus = wt_cus();
  int best = 1;
  int64_t best_cost = INT64_MAX;
  for (int S = 1; S <= 4; S *= 2) {
    if (S > 1 && P->nk / S < 16) break;
    const int64_t units = (int64_t)tiles * S, rounds = (units + cus - 1) / cus;
    const int64_t cost = rounds * ((P->nk + S - 1) / S);
    if (cost < best_cost) {
      best_cost = cost;
      best = S;
    }
  }
  P->S = best;
  // Mixed plan: with S = 2 and more tiles than CUs, the first `cus` tiles run unsplit (one full-K unit each) and only
  // the rest in two pieces, when those pieces fit one per workgroup: every workgroup then runs one full unit and at
  // most one half -- the uniform plan's three halves -- with a third of its fix-ups (the split tiles' slabs written and
  // read back).  The 8-block decoder batch: 384 tiles = 256 unsplit + 128 split.  AW_WGRAD_MIXED=0: uniform plan.
  static const bool mixed = [] { const char* e = getenv("AW_WGRAD_MIXED"); return !(e && atoi(e) == 0); }();
  P->big = (mixed && best == 2 && tiles > cus && 2 * (tiles - cus) <= cus) ? cus : 0;
  P->units = P->big + (tiles - P->big) * best;
  P->G = std::min(cus, P->units);
  P->alpha = a0.alpha;
  return AW_OK;
}

}  // namespace

namespace awg {

// The grouped decoder k = 3 weight gradient on the ping-pong kernel when the shape allows it; false -> the caller
// runs the generic grouped GEMM.
bool wgrad_conv3_try(const aw_gemm_args* args, int n, hipStream_t s) {
  const aw_gemm_args& a = args[0];
  if (g_policy < 0) return false;
  const int cin = a.conv_cin;
  const bool shape = a.a_dtype == AW_BF16 && a.a_trans && a.b_trans && cin > 0 && a.conv_operand == 1 &&
                     a.N == 3 * cin && a.M % W3_BM == 0 && cin % W3_CB == 0 && a.K % W3_BK == 0 && a.K > 0 &&
                     (a.conv_seg == 8 || a.conv_seg == 16 || a.conv_seg == 32) && a.accumulate && a.beta == 0.f &&
                     a.c_dtype == AW_F32 && a.lda % 8 == 0 && a.ldb % 8 == 0;
  if (!shape) return false;
  const int tiles = (a.M / W3_BM) * (cin / W3_CB);
  if (g_policy == 0 && tiles * n < 128) return false;   // too few tiles to fill the chip without split-K
  const int64_t ea = ((int64_t)a.K - 1) * a.lda + a.M, eb = ((int64_t)a.K - 1) * a.ldb + cin;
  if (ea * 2 >= 0x7FFFFFF0 || eb * 2 >= 0x7FFFFFF0) return false;
  W3Params P;
  memset(&P, 0, sizeof(P));
  P.M = a.M;
  P.cin = cin;
  P.K = a.K;
  P.seg = a.conv_seg;
  P.ngroups = n;
  P.tiles_m = a.M / W3_BM;
  P.tiles_i = cin / W3_CB;
  P.nblocks = tiles * n;
  P.lda = (int)a.lda;
  P.ldb = (int)a.ldb;
  P.ldc = (int)a.ldc;
  P.col_mod = a.col_mod;
  P.col_mul = a.col_mul;
  P.col_off = a.col_off;
  P.alpha = a.alpha;
  for (int g = 0; g < n; ++g) {
    P.A[g] = args[g].A;
    P.B[g] = args[g].B;
    P.C[g] = reinterpret_cast<float*>(args[g].C);
    P.rowsum[g] = args[g].a_rowsum;
  }
  hipLaunchKernelGGL(wgrad_conv3_kernel, dim3(P.nblocks), dim3(W3_NTH), 0, s, P);
  return true;
}

}  // namespace awg

extern "C" int aw_gemm_set_wgrad_policy(int mode) {
  AW_REQUIRE(mode >= -1 && mode <= 1, "aw_gemm_set_wgrad_policy: mode must be -1, 0 or 1");
  g_policy = mode;
  return AW_OK;
}


// ----------------------------------------------------------------------------------------- batched 1-tap wgrad
extern "C" int64_t aw_wgrad_batch_workspace(const aw_gemm_args* args, int n) {
  WTParams P;
  if (wt_plan(args, n, &P) != AW_OK) return -1;
  return P.S > 1 ? (int64_t)P.units * WT_SLAB * (int64_t)sizeof(float) : 16;
}

extern "C" int aw_wgrad_batch(const aw_gemm_args* args, int n, void* ws, int64_t ws_bytes, void* stream) {
  WTParams P;
  if (int st = wt_plan(args, n, &P)) return st;
  AW_REQUIRE(ws && ((uintptr_t)ws % 16) == 0 &&
                 ws_bytes >= (P.S > 1 ? (int64_t)P.units * WT_SLAB * (int64_t)sizeof(float) : 16),
             "aw_wgrad_batch: workspace must be 16-B aligned and hold aw_wgrad_batch_workspace() bytes");
  P.ws = reinterpret_cast<float*>(ws);
  P.spin = g_wt_spin;
  hipLaunchKernelGGL(wgrad_tt_kernel, dim3(P.G), dim3(WT_NTH), 0, reinterpret_cast<hipStream_t>(stream), P);
  return aw::check_launch("aw_wgrad_batch");
}

extern "C" int aw_wgrad_set_spin_limit(int polls) {
  AW_REQUIRE(polls >= 0, "aw_wgrad_set_spin_limit: polls must be >= 0");
  g_wt_spin = polls;
  return AW_OK;
}

