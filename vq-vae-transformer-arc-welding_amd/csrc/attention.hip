// Causal self-attention on MFMA for bf16 operands, head size 64 (model/transformer_block.py:37-63 at the
// transformer configs: d_model 512 / 8 heads).  Flash-style: the T x T matrices never reach HBM; the forward
// keeps the running max / sum per query and saves lse = ln sum_j exp(q.k_j / sqrt(hs)); the backward recomputes
// P from it.
//
// All products use v_mfma_f32_32x32x16_bf16.  Its 32x32 f32 result X has the COLUMN on the lane (r = lane & 31)
// and rows 8*(i>>2) + 4*h + (i&3) in register i (h = lane >> 5), so a following MFMA that sums over X's row
// index takes X straight from the registers as its B operand: k-step s of that product uses registers
// 8s..8s+7, element j <-> row 16s + 8(j>>2) + 4h + (j&3) of X; its A operand supplies the same permuted k order,
// read with ds_read_b64_tr_b16 (4 consecutive LDS rows per read).
//
//   forward (query on the lane):  S^T = K.Q^T       softmax over the rows (keys) -> P^T
//                                 O^T += V^T.P^T    (V^T via transposed reads of the V tile)
//   dQ      (query on the lane):  S^T = K.Q^T, dP^T = V.dO^T, dS^T = P^T (dP^T - delta)
//                                 dQ^T += K^T.dS^T
//   dK, dV  (key on the lane):    S = Q.K^T, dP = dO.V^T, dS = P (dP - delta)
//                                 dV^T += dO^T.P,  dK^T += Q^T.dS
//
// Tiles of 64 rows x 64 head dims (128-byte rows) are staged in LDS in one image that serves both the 16-byte
// row reads (A operands) and the transposed reads: 16-byte chunk c of row r lives at chunk c ^ f(r),
// f(r) = ((r >> 1) & 1) << 2 | ((r >> 2) & 3) -- conflict-free for both kinds of read (checked against the
// ds_read_b128 lane groups and the 32-lane halves of ds_read_b64_tr_b16).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int HS = 64;       // head size served here
constexpr int ROWB = 128;    // bytes per LDS row (64 bf16)
constexpr int TILE = 64;     // rows per staged tile
constexpr int WROWS = 32;    // rows (queries or keys) per wave
constexpr int BLK = 128;     // rows per workgroup (4 waves)
constexpr int IMG = TILE * ROWB;

// One-dimensional grid of nqb * nh * B workgroups in row-block-major order: every (b, h)'s block x = 0 (the longest
// causal range: the last query block in the forward and dQ, the first key block in dK/dV) is dispatched before any
// x = 1, so the longest workgroups start first and the short ones fill the tail.  Same-box A/B at 51 x 321 against
// the (b, h)-major order with the row blocks of one head on one XCD (their K/V re-reads shared in L2): forward
// 24.9 -> 23.2 us, backward 81.7 -> 80.1 us (tools/attn_ab.sh).
struct BlockId {
  int x, h, b;
  __device__ __forceinline__ BlockId(int nqb, int nh) {
    const int nbh = (int)gridDim.x / nqb, bid = (int)blockIdx.x;
    x = bid / nbh;
    const int bh = bid % nbh;
    h = bh % nh;
    b = bh / nh;
  }
};

__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int img_off(int r, int c) { return r * ROWB + ((c ^ swz(r)) << 4); }

__device__ __forceinline__ f32x16 mfma32(const uint4& a, const uint4& b, const f32x16& c) {
  bf16x8 av, bv;
  memcpy(&av, &a, 16);
  memcpy(&bv, &b, 16);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// 16-byte A/B fragment of row `r` for k-step `ks` (head dims 16ks + 8h .. +7)
__device__ __forceinline__ uint4 row_frag(const char* img, int r, int ks, int h) {
  return *reinterpret_cast<const uint4*>(img + img_off(r, 2 * ks + h));
}

// Transposed fragment: A operand of a product summing over the tile's rows, k-step covering rows
// rb + {0..3} and rb + 8 + {0..3} (rb = 16 s + 4 h), columns (head dims) 32 dt + (lane & 31).
__device__ __forceinline__ uint4 tr_frag(const char* img, int rb, int dt, int lane) {
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = 32 * dt + 16 * (G & 1) + 4 * p;       // head dim of the 4 elements this lane addresses
  const int c = col >> 3, within = (col & 7) * 2;
  const int r0 = rb + q, r1 = rb + 8 + q;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(uintptr_t)(img + img_off(r0, c) + within));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(uintptr_t)(img + img_off(r1, c) + within));
  uint4 out;
  memcpy(&out, &lo, 8);
  memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
  return out;
}

// Registers 8s..8s+7 of an accumulator as a bf16 B fragment
__device__ __forceinline__ uint4 pack8(const f32x16& a, int s) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)a[8 * s + j];
  uint4 u;
  memcpy(&u, &v, 16);
  return u;
}

// Global -> registers for one 64-row tile (rows r0.., row stride ld elements, column offset col0); rows >= T
// are zero.  Thread t carries chunks t and t + 256 of the 512.
struct TileRegs {
  uint4 v[2];
};
__device__ __forceinline__ void tile_load(TileRegs& tr, const bf16* src, int64_t ld, int col0, int r0, int T_,
                                          int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
    const int gr = r0 + row;
    tr.v[u] = gr < T_ ? *reinterpret_cast<const uint4*>(src + (int64_t)gr * ld + col0 + ch * 8) : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void tile_store(const TileRegs& tr, char* img, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(img + img_off(row, ch)) = tr.v[u];
  }
}

// A wave's 32 rows x 64 head dims (an accumulator pair with the row on the lane, the dims in the registers) stored as
// whole 128-byte rows: the fragments go to the wave's own 4 KB of LDS (16-byte chunks XOR-swizzled by row), then
// every lane writes 16-byte chunks, 8 lanes per row.  Stored straight from the registers, each 8-byte wave store
// touched 32 rows at a 128-byte stride (MI355X_MICROARCH.md: a store-issue-bound tail).
__device__ __forceinline__ void store_rows(const f32x16 (&a)[2], float s, char* reg, bf16* out0, int64_t ld,
                                           int nrows, int lane) {
  const int r = lane & 31, hf = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      bf16 v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (bf16)(a[dt][4 * g4 + e] * s);
      uint2 u;
      memcpy(&u, v, 8);
      *reinterpret_cast<uint2*>(reg + r * ROWB + (((4 * dt + g4) ^ (r & 7)) << 4) + 8 * hf) = u;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (lane >> 3) + 8 * j, c = lane & 7;
    if (row < nrows) {
      const uint4 u = *reinterpret_cast<const uint4*>(reg + row * ROWB + ((c ^ (row & 7)) << 4));
      // non-temporal, as the GEMM epilogues: the next launch reads them (decoder step 5.314 / 5.315 / 5.315 ->
      // 5.306 / 5.309 / 5.300 ms against ordinary stores, same box)
      __builtin_nontemporal_store(__builtin_bit_cast(aw_v4i32, u), reinterpret_cast<aw_v4i32*>(out0 + row * ld + 8 * c));
    }
  }
}

__device__ __forceinline__ void store4_bf16(bf16* dst, const f32x16& a, int g4, float s) {
  bf16 v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (bf16)(a[4 * g4 + e] * s);
  uint2 u;
  memcpy(&u, v, 8);
  *reinterpret_cast<uint2*>(dst) = u;
}

// ---------------------------------------------------------------- forward
// grid (ceil(T/128), n_head, B), 256 threads; wave w owns queries qb*128 + 32w .. +31.
__global__ __launch_bounds__(256, 2) void attn_fwd_mfma_kernel(const bf16* __restrict__ qkv, int T_, int nh, int d,
                                                            bf16* __restrict__ y, float* __restrict__ lse,
                                                            float c2, float scale) {
  // K/V images double-buffered (tile t in buffer t & 1): storing tile t cannot race the reads of tile t - 1, so one
  // barrier per tile publishes it
  __shared__ __attribute__((aligned(16))) char KV[4 * IMG];
  const int nqb = (T_ + BLK - 1) / BLK;
  const BlockId id(nqb, nh);
  const int qb = nqb - 1 - id.x;  // longest key ranges first
  const int h = id.h, b = id.b;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hf = lane >> 5;
  const int64_t ld = 3 * (int64_t)d;
  const bf16* base = qkv + (int64_t)b * T_ * ld;
  const int qw = qb * BLK + w * WROWS, q = qw + r;
  const int qc = min(q, T_ - 1);
  uint4 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const uint4*>(base + (int64_t)qc * ld + h * HS + 16 * s + 8 * hf);
  f32x16 o[2] = {zero16(), zero16()};
  float m = -__builtin_huge_valf(), l = 0.f;
  const int kend = min(T_, qb * BLK + BLK);
  const int nt = (kend + TILE - 1) / TILE;
  TileRegs kr, vr;
  tile_load(kr, base, ld, d + h * HS, 0, T_, tid);
  tile_load(vr, base, ld, 2 * d + h * HS, 0, T_, tid);
  for (int t = 0; t < nt; ++t) {
    const int k0 = t * TILE;
    char* Ks = KV + (t & 1) * 2 * IMG;
    char* Vs = Ks + IMG;
    tile_store(kr, Ks, tid);
    tile_store(vr, Vs, tid);
    // the next tile's loads go out before the barrier: their latency runs under the barrier wait too
    if (t + 1 < nt) {
      tile_load(kr, base, ld, d + h * HS, k0 + TILE, T_, tid);
      tile_load(vr, base, ld, 2 * d + h * HS, k0 + TILE, T_, tid);
    }
    __syncthreads();
    if (k0 > qw + WROWS - 1) continue;  // wave-uniform: the whole tile lies after this wave's queries
    f32x16 s[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      s[st] = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s[st] = mfma32(row_frag(Ks, 32 * st + r, ks, hf), qf[ks], s[st]);
    }
    const bool edge = (k0 + TILE - 1 > qw) || (k0 + TILE > T_);
    // causal / length mask as selects against one per-lane limit, only on the (wave-uniform) edge tiles: the empty
    // asm keeps the branch -- if-converted, the 64 compares + selects ran on every tile (a third of the loop's VALU)
    if (edge) {
      asm volatile("" ::: "memory");
      const int lim = min(q, T_ - 1) - (k0 + 4 * hf);
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          s[st][i] = (32 * st + 8 * (i >> 2) + (i & 3) > lim) ? -__builtin_huge_valf() : s[st][i];
    }
    float mx = -__builtin_huge_valf();
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[st][i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    // the running max moves only when some lane's grows by more than 2^8 in P: below that the stale max keeps
    // every P <= 256 (same products, other roundings) and the rescale of o and l is skipped (wave-uniform)
    const bool resc = __builtin_amdgcn_ballot_w64((mn - m) * c2 > 8.f) != 0;
    float alpha = 1.f;
    if (resc) {
      alpha = __builtin_amdgcn_exp2f((m - mn) * c2);
      m = mn;
    }
    const float mc = m * c2;
    // exponent arguments and the row sum as f32 pairs (v_pk_fma_f32 / v_pk_add_f32)
    f32x2 ls2 = {0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 a = __builtin_elementwise_fma((f32x2){s[st][i], s[st][i + 1]}, (f32x2){c2, c2}, (f32x2){-mc, -mc});
        const f32x2 p = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
        s[st][i] = p.x;
        s[st][i + 1] = p.y;
        ls2 += p;
      }
    if (resc) {
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
    }
    l += ls2.x + ls2.y;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 pb = pack8(s[st], s2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) o[dt] = mfma32(tr_frag(Vs, 32 * st + 16 * s2 + 4 * hf, dt, lane), pb, o[dt]);
      }
  }
  l += __shfl_xor(l, 32, 64);
  // 1 / l per lane: lanes past T carry l = 0 (every score masked); their rows are not stored
  const float inv = q < T_ ? 1.f / l : 0.f;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] *= inv;
  if (q < T_ && hf == 0) lse[((int64_t)b * nh + h) * T_ + q] = m * scale + logf(l);
  __syncthreads();   // every wave's reads of the K / V images are done: the images become store staging
  if (qw < T_)
    store_rows(o, 1.f, KV + w * 4096, y + ((int64_t)b * T_ + qw) * d + h * HS, d, min(WROWS, T_ - qw), lane);
}

// ---------------------------------------------------------------- backward: LDS-DMA tile ring
// The two backward kernels take every tile by LDS-DMA (buffer_load_dwordx4 ... lds: lane l of a wave-instruction
// writes the 16 bytes at M0 + 16 l) into a ring NB tiles deep, so a workgroup keeps NB - 1 tiles of reads in flight
// under its MFMA / softmax work; no staging VGPRs, no ds_write.  A piece is 1 KiB = 8 rows of a 64-row image; the
// swizzle is applied on the SOURCE address (LDS slot c of row r holds chunk c ^ swz(r)), and rows past the end of
// the sequence come back as zeros from the buffer range check.  Same-box A/B at 51 x 321 against the register-staged
// double buffer: dQ + dK/dV 80.1 -> 76.5 us.  (The forward measured slower on the ring, 26.0 vs 23.2 us: at 80 KB of
// LDS it runs two workgroups per CU instead of three, and with its loads alone -- no MFMA, no softmax -- the
// register-staged forward already takes 19.7 us, so it is bound by the load pipeline, not by its depth.)
constexpr int NB = 3;          // ring depth (tiles)
constexpr int SLOT = 2 * IMG;  // one ring slot: two 64-row images

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
// source byte offset of lane `lane` in piece jj of a 64-row image whose rows are ldb bytes apart
__device__ __forceinline__ int piece_off(int jj, int lane, int ldb) {
  const int row = 8 * jj + (lane >> 3);
  return row * ldb + (((lane & 7) ^ swz(row)) << 4);
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// dQ on the ring.  Wave w fills bytes [4 KiB w, 4 KiB w + 4 KiB) of every slot: K rows 32w.. (w < 2) or V
// rows 32(w - 2).. (w >= 2).  The stationary operands of a wave are its own 32 rows only: Q is staged where nothing
// but that wave's own later DMA lands (bytes [4 KiB w, +4 KiB) of slot NB - 1: a 128-row image over the slot; the
// wave's first DMA into it follows its reads); dO and O go straight to registers (the dO fragments are the B operand
// of dP^T as they are; O only meets dO in delta_i = dO_i . O_i, which the wave writes after its loop for the dK/dV
// launch).  48 KB of LDS: three workgroups per CU (the dO / O images of round 3 held it to two at 80 KB).
__global__ __launch_bounds__(256, 2) void attn_dq_ring_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dy,
                                                           const bf16* __restrict__ y, const float* __restrict__ lse,
                                                           float* __restrict__ delta, int T_, int nh, int d,
                                                           bf16* __restrict__ dqkv, float c2, float scale) {
  __shared__ __attribute__((aligned(16))) char L[NB * SLOT];   // the K / V ring (Q of the own rows in slot NB - 1)
  const int nqb = (T_ + BLK - 1) / BLK;
  const BlockId id(nqb, nh);
  const int qb = nqb - 1 - id.x;
  const int h = id.h, b = id.b;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ldb = 6 * d;   // bytes per qkv row
  const char* bbase = reinterpret_cast<const char*>(qkv) + (int64_t)b * T_ * ldb;
  const uint32_t lring = aw_lds_addr(L);
  const int q0 = qb * BLK, qw = q0 + w * WROWS, q = qw + r;
  const int kend = min(T_, q0 + BLK);
  const int nt = (kend + TILE - 1) / TILE;
  const int sel = w >> 1;   // 0: K image, 1: V image
  int off[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) off[u] = piece_off(4 * (w & 1) + u, lane, ldb);
  // dO and O of the lane's row (clamped past T: those rows are never stored), 16 B per k-step as row_frag reads;
  // issued before the DMAs so that the counted waits below cover them
  uint4 qf[4], gf[4], yf[4];
  {
    const int qc = min(q, T_ - 1);
    const bf16* grow = dy + ((int64_t)b * T_ + qc) * d + h * HS + 8 * hf;
    const bf16* yrow = y + ((int64_t)b * T_ + qc) * d + h * HS + 8 * hf;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      gf[s] = *reinterpret_cast<const uint4*>(grow + 16 * s);
      yf[s] = *reinterpret_cast<const uint4*>(yrow + 16 * s);
    }
  }
  {   // own rows of Q (LDS-DMA)
    const aw_v4i32 dq = aw_rdesc(bbase + (int64_t)q0 * ldb + h * HS * 2, (uint32_t)(T_ - q0) * ldb);
    const uint32_t sq = lring + (NB - 1) * SLOT;
#pragma unroll
    for (int u = 0; u < 4; ++u) aw_dma16(sq + (4 * w + u) * 1024, piece_off(4 * w + u, lane, ldb), dq);
  }
  auto issue = [&](int t) {
    const int k0 = t * TILE;
    const uint32_t nrec = t < nt ? (uint32_t)(T_ - k0) * ldb : 0u;
    const aw_v4i32 ds = aw_rdesc(bbase + (int64_t)k0 * ldb + ((1 + sel) * d + h * HS) * 2, nrec);
    const uint32_t s = lring + (t % NB) * SLOT + 4096 * w;
#pragma unroll
    for (int u = 0; u < 4; ++u) aw_dma16(s + 1024 * u, off[u], ds);
  };
#pragma unroll
  for (int t = 0; t < NB - 1; ++t) issue(t);
  aw_vm_wait<4 * (NB - 2)>();   // dO / O, the Q pieces and ring tile 0 landed
  raw_barrier();
  float Dl = 0.f;
  {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 yv = __builtin_bit_cast(bf16x8, yf[s]);
      const bf16x8 gv = __builtin_bit_cast(bf16x8, gf[s]);
#pragma unroll
      for (int e = 0; e < 8; ++e) Dl = fmaf((float)gv[e], (float)yv[e], Dl);
    }
    Dl += __shfl_xor(Dl, 32, 64);
  }
  {
    const char* Qs = L + (NB - 1) * SLOT;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = row_frag(Qs, 32 * w + r, s, hf);
    lgkm_wait0();   // the Q reads retire before this wave's DMA of tile NB - 1 overwrites them
  }
  const int64_t st_i = ((int64_t)b * nh + h) * T_ + min(q, T_ - 1);
  const float L2 = lse[st_i] * 1.4426950408889634f;
  f32x16 acc[2] = {zero16(), zero16()};
  const bool active = qw < T_;
  for (int t = 0; t < nt; ++t) {
    if (t > 0) {
      aw_vm_wait<4 * (NB - 2)>();
      raw_barrier();
    }
    issue(t + NB - 1);
    const int k0 = t * TILE;
    if (!active || k0 > qw + WROWS - 1) continue;
    const char* Ks = L + (t % NB) * SLOT;
    const char* Vs = Ks + IMG;
    const bool edge = (k0 + TILE - 1 > qw) || (k0 + TILE > T_);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      // keys k0+32.. lie after every query of the wave (or past T) on its diagonal tile: nothing to add
      if (st == 1 && (k0 + 32 > qw + WROWS - 1 || k0 + 32 >= T_)) break;   // wave-uniform
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s = mfma32(row_frag(Ks, 32 * st + r, ks, hf), qf[ks], s);
        dp = mfma32(row_frag(Vs, 32 * st + r, ks, hf), gf[ks], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = __builtin_amdgcn_exp2f(fmaf(s[i], c2, -L2));
      if (edge) {
        asm volatile("" ::: "memory");
        const int lim = min(q, T_ - 1) - (k0 + 32 * st + 4 * hf);
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = (8 * (i >> 2) + (i & 3) > lim) ? 0.f : s[i];
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = s[i] * (dp[i] - Dl);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 db = pack8(s, s2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) acc[dt] = mfma32(tr_frag(Ks, 32 * st + 16 * s2 + 4 * hf, dt, lane), db, acc[dt]);
      }
    }
  }
  aw_vm_wait<0>();
  if (q < T_ && hf == 0) delta[st_i] = Dl;
  raw_barrier();   // every wave's reads of the ring are done; bytes [4 KiB w, +4 KiB) of slot 0 take only w's DMAs
  if (qw < T_)
    store_rows(acc, scale, L + 4096 * w, dqkv + ((int64_t)b * T_ + qw) * (3 * (int64_t)d) + h * HS, 3 * (int64_t)d,
               min(WROWS, T_ - qw), lane);
}

// dK, dV on the ring, key-stationary.  A slot holds the query tile's Q image, dO image, lse row and
// delta row; wave w fills bytes [4 KiB w, +4 KiB) of the two images (Q rows 32w.. for w < 2, dO rows 32(w - 2)..
// for w >= 2) and one 256-byte row (lse for even w, delta for odd w: two waves load each row, the same bytes), so
// every wave issues five pieces per tile.  The wave's own K rows are staged in slot NB - 1 (as Q in the dQ kernel),
// its V rows go straight to registers (they are only ever the B operand of dP).  49.5 KB of LDS and at most 168
// VGPRs: three workgroups per CU (round 3: 65.5 KB and 202 VGPRs, two).
constexpr int DSLOT = 2 * IMG + 2 * TILE * 4;
__global__ __launch_bounds__(256, 3) void attn_dkv_ring_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dy,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta, int T_, int nh, int d,
                                                            bf16* __restrict__ dqkv, float c2, float scale) {
  __shared__ __attribute__((aligned(16))) char L[NB * DSLOT];
  const BlockId id((T_ + BLK - 1) / BLK, nh);
  const int kb = id.x;
  const int h = id.h, b = id.b;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ldb = 6 * d, ldg = 2 * d;
  const char* bbase = reinterpret_cast<const char*>(qkv) + (int64_t)b * T_ * ldb;
  const char* gbase = reinterpret_cast<const char*>(dy) + (int64_t)b * T_ * ldg;
  const uint32_t lring = aw_lds_addr(L);
  const int k0b = kb * BLK, kw = k0b + w * WROWS, key = kw + r;
  const int qstart = k0b;   // BLK is a multiple of TILE
  const int nqt = (T_ - qstart + TILE - 1) / TILE;
  const int sel = w >> 1;   // 0: Q image, 1: dO image
  const int lds_src = sel ? ldg : ldb;
  int off[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) off[u] = piece_off(4 * (w & 1) + u, lane, lds_src);
  const int64_t sbase = ((int64_t)b * nh + h) * T_;
  const float* vec = (w & 1) ? delta : lse;
  // V of the lane's key row to registers (clamped past T: those keys are never stored), issued before the DMAs
  uint4 kf[4], vf[4];
  {
    const bf16* vrow = qkv + ((int64_t)b * T_ + min(key, T_ - 1)) * (3 * (int64_t)d) + 2 * d + h * HS + 8 * hf;
#pragma unroll
    for (int s = 0; s < 4; ++s) vf[s] = *reinterpret_cast<const uint4*>(vrow + 16 * s);
  }
  {   // own rows of K (into slot NB - 1)
    const aw_v4i32 dk = aw_rdesc(bbase + (int64_t)k0b * ldb + (d + h * HS) * 2, (uint32_t)(T_ - k0b) * ldb);
    const uint32_t sk = lring + (NB - 1) * DSLOT;
#pragma unroll
    for (int u = 0; u < 4; ++u) aw_dma16(sk + (4 * w + u) * 1024, piece_off(4 * w + u, lane, ldb), dk);
  }
  auto issue = [&](int i) {
    const int q0 = qstart + TILE * i;
    const bool valid = i < nqt;
    const char* src = sel ? gbase + (int64_t)q0 * ldg + h * HS * 2 : bbase + (int64_t)q0 * ldb + h * HS * 2;
    const aw_v4i32 ds = aw_rdesc(src, valid ? (uint32_t)(T_ - q0) * lds_src : 0u);
    const aw_v4i32 dvv = aw_rdesc(reinterpret_cast<const char*>(vec + sbase + q0), valid ? (uint32_t)(T_ - q0) * 4 : 0u);
    const uint32_t s = lring + (i % NB) * DSLOT;
#pragma unroll
    for (int u = 0; u < 4; ++u) aw_dma16(s + 4096 * w + 1024 * u, off[u], ds);
    aw_dma4(s + 2 * IMG + (w & 1) * (TILE * 4), lane * 4, dvv);
  };
#pragma unroll
  for (int i = 0; i < NB - 1; ++i) issue(i);
  aw_vm_wait<5 * (NB - 2)>();
  raw_barrier();
  {
    const char* Ksg = L + (NB - 1) * DSLOT;
#pragma unroll
    for (int s = 0; s < 4; ++s) kf[s] = row_frag(Ksg, 32 * w + r, s, hf);
    lgkm_wait0();
  }
  f32x16 dk[2] = {zero16(), zero16()}, dv[2] = {zero16(), zero16()};
  const bool active = kw < T_;
  for (int i = 0; i < nqt; ++i) {
    if (i > 0) {
      aw_vm_wait<5 * (NB - 2)>();
      raw_barrier();
    }
    issue(i + NB - 1);
    const int q0 = qstart + TILE * i;
    if (!active || q0 + TILE - 1 < kw) continue;
    const char* Qs = L + (i % NB) * DSLOT;
    const char* Gs = Qs + IMG;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * IMG);
    const float* Ds = Ls + TILE;
    const bool edge = (q0 < kw + WROWS - 1) || (q0 + TILE > T_);
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      // queries q0+32qs.. all precede the wave's first key (or lie past T): every P of the sub-tile is masked
      if (q0 + 32 * qs + 31 < kw || q0 + 32 * qs >= T_) continue;   // wave-uniform
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s = mfma32(row_frag(Qs, 32 * qs + r, ks, hf), kf[ks], s);
        dp = mfma32(row_frag(Gs, 32 * qs + r, ks, hf), vf[ks], dp);
      }
      f32x16 p;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int ql = 32 * qs + 8 * g4 + 4 * hf;
        const float4 L4 = *reinterpret_cast<const float4*>(Ls + ql);
        const float Lv[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          p[4 * g4 + e] = __builtin_amdgcn_exp2f(fmaf(s[4 * g4 + e], c2, -Lv[e] * 1.4426950408889634f));
      }
      if (edge) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int qq = q0 + 32 * qs + 8 * (e >> 2) + 4 * hf + (e & 3);
          p[e] = (qq < key || qq >= T_) ? 0.f : p[e];
        }
      }
      // dS = P (dP - delta): the delta rows are read from the slot per 4-row group (no 16-register copy)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 D4 = *reinterpret_cast<const float4*>(Ds + 32 * qs + 8 * g4 + 4 * hf);
        const float Dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) s[4 * g4 + e] = p[4 * g4 + e] * (dp[4 * g4 + e] - Dv[e]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const uint4 pb = pack8(p, s2), db = pack8(s, s2);
        const int rb = 32 * qs + 16 * s2 + 4 * hf;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma32(tr_frag(Gs, rb, dt, lane), pb, dv[dt]);
          dk[dt] = mfma32(tr_frag(Qs, rb, dt, lane), db, dk[dt]);
        }
      }
    }
  }
  aw_vm_wait<0>();
  raw_barrier();   // every wave's reads of the ring are done; bytes [4 KiB w, +4 KiB) of a slot take only w's DMAs
  if (kw < T_) {
    bf16* out = dqkv + ((int64_t)b * T_ + kw) * (3 * (int64_t)d) + h * HS;
    const int n = min(WROWS, T_ - kw);
    store_rows(dk, scale, L + 4096 * w, out + d, 3 * (int64_t)d, n, lane);
    store_rows(dv, 1.f, L + DSLOT + 4096 * w, out + 2 * d, 3 * (int64_t)d, n, lane);
  }
}


}  // namespace

namespace aw {

// The backward's LDS-DMA buffer offsets are 32-bit: one sequence of qkv rows must stay under 2 GiB.
bool attn_mfma_supported(int dtype, int hs, int d, int64_t T) {
  return dtype == AW_BF16 && hs == HS && d % 8 == 0 && T * 6 * (int64_t)d < (1ll << 31);
}

void attn_fwd_mfma(const void* qkv, int64_t B, int T, int nh, int d, void* y, float* lse, hipStream_t s) {
  const float scale = 1.0f / sqrtf((float)HS);
  dim3 grid((unsigned)(((T + BLK - 1) / BLK) * (int64_t)nh * B));
  hipLaunchKernelGGL(attn_fwd_mfma_kernel, grid, dim3(256), 0, s, (const bf16*)qkv, T, nh, d, (bf16*)y, lse,
                     scale * 1.4426950408889634f, scale);
}

void attn_bwd_mfma(const void* qkv, const void* y, const void* dy, const float* lse, float* delta, int64_t B, int T,
                   int nh, int d, void* dqkv, hipStream_t s) {
  const float scale = 1.0f / sqrtf((float)HS);
  dim3 grid((unsigned)(((T + BLK - 1) / BLK) * (int64_t)nh * B));
  hipLaunchKernelGGL(attn_dq_ring_kernel, grid, dim3(256), 0, s, (const bf16*)qkv, (const bf16*)dy, (const bf16*)y,
                     lse, delta, T, nh, d, (bf16*)dqkv, scale * 1.4426950408889634f, scale);
  hipLaunchKernelGGL(attn_dkv_ring_kernel, grid, dim3(256), 0, s, (const bf16*)qkv, (const bf16*)dy, lse, delta, T,
                     nh, d, (bf16*)dqkv, scale * 1.4426950408889634f, scale);
}

}  // namespace aw
