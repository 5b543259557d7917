// Vector quantizer (model/vector_quantizer.py:59-131) for gfx950.
//
// Forward: register-blocked distance tiles with the codebook streamed through LDS (see vq_fwd_kernel).
// Distances follow the reference expression exactly in fp32:
//     d_k = fl( fl(|z|^2 + |e_k|^2) - 2 * dot(z, e_k) ),  dot = k-ordered fmaf chain over the embedding dim
// (torch's CPU sgemm on this shape is bit-identical to that chain -- measured), so the
// argmin (lexicographic (d, k) minimum == torch.argmin first-index tie rule) is bit-exact.
// No MFMA (the north-star design): fp32 VALU, whose rate equals the f32-input MFMA's on gfx950.
#include <stdlib.h>

#include "common.h"

namespace {

// ---------------------------------------------------------------- forward: register-blocked distance tiles
// One workgroup = 64 rows (the z tile stays in LDS for the whole launch) x 8 waves (two per SIMD).  The codebook
// streams through LDS in code tiles of 512 codes (64 per wave) x 16-float chunks of the embedding dim, stored
// d-major ([d][code]) and register-prefetched one chunk ahead.  Lane (lr, lc) = (lane >> 3, lane & 7) of wave w
// owns the 8 x 8 outer-product block rows {lr + 8i} x codes {64w + 8lc + j}: per embedding index it holds the
// 8 code values as 4 register pairs and issues 32 packed FMAs (v_pk_fma_f32: the row value in both halves,
// a pair of codes) -- the FP32 vector peak needs the packed form (a scalar v_fmac loop tops out near 70 TF,
// tools/probe/valu_fma_probe.hip).  Per 4-deep step: 8 z reads (row broadcasts) + 8 e reads + 128 v_pk_fma.
// Each (row, code) accumulator is the reference's dot product as an in-order fused-multiply-add chain over the
// embedding dim; |z|^2 and |e_k|^2 are in-order sums of squares; the distance is fl(fl(|z|^2 + |e_k|^2) - 2 * dot)
// and the argmin the lexicographic (d, k) minimum (torch.argmin's first-index tie rule).  The register footprint
// does not depend on D, so the stress codebook (K 8192 x D 256) runs at the same occupancy.

constexpr int VQ_THREADS = 512;
constexpr int VQ_CODES = 512;
constexpr int VQ_DC = 16;           // embedding floats per staged chunk

// Code counts are gathered per workgroup in LDS, not added per row: isolated at the configs[1] shape 39.1 -> 28.0 us
// (a build without the count atomics: 26.4 us; round-4 probes).

template <int D, int ROWS> struct VqLds {
  static constexpr int ZP = D + 4;                                   // z image pitch (disjoint banks per row)
  static constexpr int Z = ROWS * ZP;                                // floats
  static constexpr int EP = VQ_CODES + 4;                            // [d][code] pitch: a staging store's 4 dims
                                                                     // of a code land on 2-way (free) banks
  static constexpr int E = VQ_DC * EP;                               // floats per stage, [d][code]
  static constexpr int TOTAL = Z + 2 * E + 2 * VQ_CODES + ROWS;      // + ee[2][512] + zz[ROWS]
};

// (bd, bk) <- (d, k) when ok and (d, k) < (bd, bk) lexicographically (torch.argmin's first-index tie rule; a NaN d
// is never taken).  Branch-free selects: written as `if (a || (b && c)) {...}` the compiler made an exec-mask branch
// of every comparison (155 saveexec / 50 branches in the pinned kernel's argmin, which then took longer than the
// distance loop).
__device__ __forceinline__ void lex_take(float d, int k, bool ok, float& bd, int& bk) {
  const bool t = ok & ((d < bd) | ((d == bd) & (k < bk)));
  bd = t ? d : bd;
  bk = t ? k : bk;
}

// The end of a forward workgroup of ROWS = 8 RPL rows: each lane holds the lexicographic (d, k) minimum of its
// (row lr + 8i, 8 codes) blocks; the argmin across the 8 code lanes of a row group, then across the 8 waves (LDS
// `scratch`, free by now), then z_q / idx / counts / sqerr.
template <int D, int RPL>
__device__ __forceinline__ void vq_finish(float (&best)[RPL], int (&bestk)[RPL], float* scratch, int hcap,
                                          const float* zs, double* red, const float* __restrict__ E, int64_t N, int K,
                                          int64_t row0, float* __restrict__ zq, int64_t* __restrict__ idx,
                                          float* __restrict__ counts, double* __restrict__ sqerr, void* __restrict__ zq2,
                                          int zq2_bf16) {
  constexpr int ROWS = 8 * RPL, ZP = D + 4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane >> 3, lc = lane & 7;
  float* es = scratch;
  // ---- argmin across the 8 code lanes of a row group, then across the 8 waves (LDS, the e stages are free)
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      const float d = __shfl_xor(best[i], o, 64);
      const int k = __shfl_xor(bestk[i], o, 64);
      lex_take(d, k, true, best[i], bestk[i]);
    }
  }
  float* rd = es;                                        // [8 waves][ROWS]
  int* rk = reinterpret_cast<int*>(es + 8 * ROWS);
  if (lc == 0) {
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
      rd[w * ROWS + lr + 8 * i] = best[i];
      rk[w * ROWS + lr + 8 * i] = bestk[i];
    }
  }
  __syncthreads();
  // ---- epilogue over the whole workgroup: thread (row r, quad q) of the ROWS x D/4 float4 items resolves its
  // row's winner from the 8 wave candidates (LDS broadcast reads), gathers e_k's quad and writes z_q (+ the operand
  // copy) coalesced; the q == 0 thread of a row writes idx and counts the code.
  constexpr int DQ = D / 4;
  double se = 0.0;
  // the workgroup's code counts gather in LDS (the e stages past rd / rk are free now) and go out as one sweep of
  // the K bins: one atomic per distinct code, issued bin-contiguous, instead of one per row from the epilogue
  const int HCAP = hcap;
  float* hist = es + 16 * ROWS;
  const bool lds_counts = K <= HCAP;
  if (lds_counts) {
    for (int i = tid; i < K; i += VQ_THREADS) hist[i] = 0.f;
    __syncthreads();
  }
  for (int it = tid; it < ROWS * DQ; it += VQ_THREADS) {
    const int r = it / DQ, q = it - r * DQ;
    const int64_t row = row0 + r;
    if (row >= N) break;   // rows ascend with it
    float bd = rd[r];
    int bk = rk[r];
#pragma unroll
    for (int v = 1; v < 8; ++v) lex_take(rd[v * ROWS + r], rk[v * ROWS + r], true, bd, bk);
    if (bk < 0 || bk >= K) bk = 0;  // all-NaN row guard (torch would return the NaN position)
    if (q == 0) {
      idx[row] = bk;
      if (lds_counts)
        atomicAdd(hist + bk, 1.0f);
      else
      atomicAdd(counts + bk, 1.0f);
    }
    const float4 e = reinterpret_cast<const float4*>(E + (int64_t)bk * D)[q];
    const float4 zv = *reinterpret_cast<const float4*>(zs + r * ZP + 4 * q);
    const float d0 = __fsub_rn(e.x, zv.x), d1 = __fsub_rn(e.y, zv.y);
    const float d2 = __fsub_rn(e.z, zv.z), d3 = __fsub_rn(e.w, zv.w);
    float4 o;
    o.x = __fadd_rn(zv.x, d0);  // z + (z_q - z).detach()
    o.y = __fadd_rn(zv.y, d1);
    o.z = __fadd_rn(zv.z, d2);
    o.w = __fadd_rn(zv.w, d3);
    reinterpret_cast<float4*>(zq + row * D)[q] = o;
    if (zq2) {   // the GEMM operand copy of z_q (the decoder's first conv reads it): no separate cast launch
      if (zq2_bf16) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        reinterpret_cast<bf16x4*>(zq2)[row * DQ + q] = bf16x4{(bf16)o.x, (bf16)o.y, (bf16)o.z, (bf16)o.w};
      } else {
        reinterpret_cast<float4*>(zq2)[row * DQ + q] = o;
      }
    }
    se += (double)(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
  }
  se = wave_sum_d(se);
  if (lane == 0) red[w] = se;
  // LDS-only barrier: __syncthreads' release fence would also wait for this workgroup's z_q stores and count atomics
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (lds_counts)
    for (int i = tid; i < K; i += VQ_THREADS) {
      const float c = hist[i];
      if (c != 0.f) atomicAdd(counts + i, c);
    }
  if (tid == 0) {
    double t = 0.0;
#pragma unroll
    for (int v = 0; v < 8; ++v) t += red[v];
    atomicAdd(sqerr, t);
  }
}


// RPL = rows per lane (ROWS = 8 RPL rows per workgroup): 8 for long row counts, 4 to put two workgroups on every CU
// when N / 64 would leave the chip at one (the bench shape: N 16384 -> 512 workgroups of 32 rows)
template <int D, int RPL>
__global__ __launch_bounds__(VQ_THREADS, 2) void vq_fwd_kernel(const float* __restrict__ z,
                                                               const float* __restrict__ E, int64_t N, int K,
                                                               float* __restrict__ zq, int64_t* __restrict__ idx,
                                                               float* __restrict__ counts,
                                                               double* __restrict__ sqerr, void* __restrict__ zq2,
                                                               int zq2_bf16) {
  constexpr int ROWS = 8 * RPL;
  using L = VqLds<D, ROWS>;
  constexpr int ZP = L::ZP, ND = D / VQ_DC;
  __shared__ __attribute__((aligned(16))) float smem[L::TOTAL];
  float* zs = smem;
  float* es = smem + L::Z;                 // [2][VQ_DC][VQ_CODES]
  float* ees = es + 2 * L::E;              // [2][VQ_CODES]
  float* zzs = ees + 2 * VQ_CODES;         // [ROWS]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane >> 3, lc = lane & 7;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;

  // ---- z tile -> LDS (rows beyond N are zero), |z|^2 per row
  for (int i = tid; i < ROWS * (D / 4); i += VQ_THREADS) {
    const int r = i / (D / 4), q = i - r * (D / 4);
    const int64_t gr = row0 + r;
    const float4 v = gr < N ? reinterpret_cast<const float4*>(z + gr * D)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(zs + r * ZP + 4 * q) = v;
  }
  __syncthreads();
  if (tid < ROWS) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = __fadd_rn(s, __fmul_rn(zs[tid * ZP + d], zs[tid * ZP + d]));
    zzs[tid] = s;
  }

  // ---- codebook stream: step s = (code tile s / ND, chunk s % ND).  Staging is coalesced: float4 u of thread t
  // is quad (t & 3) of code 128u + (t >> 2) (4 lanes per 64-B chunk row, 16 cache lines per load instruction);
  // the store transposes it into the [d][code] image.  |e_k|^2 is summed in embedding order by the thread of code
  // k from the published image at the start of each step.
  constexpr int EP = L::EP;
  const int ntiles = (K + VQ_CODES - 1) / VQ_CODES;
  const int nsteps = ntiles * ND;
  float4 pre[VQ_DC / 4];
  float ee_acc = 0.f;
  auto load = [&](int st) {
    const int ct = st / ND, dc = st - ct * ND;
#pragma unroll
    for (int u = 0; u < VQ_DC / 4; ++u) {
      const int code = ct * VQ_CODES + 128 * u + (tid >> 2);
      pre[u] = code < K ? reinterpret_cast<const float4*>(E + (int64_t)code * D + dc * VQ_DC)[tid & 3]
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int st) {
    float* dst = es + (st & 1) * L::E + 4 * (tid & 3) * EP + (tid >> 2);
#pragma unroll
    for (int u = 0; u < VQ_DC / 4; ++u) {
      dst[0 * EP + 128 * u] = pre[u].x;
      dst[1 * EP + 128 * u] = pre[u].y;
      dst[2 * EP + 128 * u] = pre[u].z;
      dst[3 * EP + 128 * u] = pre[u].w;
    }
  };
  auto norms = [&](int st) {   // chunk st is published: continue this thread's code's in-order sum of squares
    const int ct = st / ND, dc = st - ct * ND;
    const float* src = es + (st & 1) * L::E + tid;
    if (dc == 0) ee_acc = 0.f;
#pragma unroll
    for (int d = 0; d < VQ_DC; ++d) ee_acc = __fadd_rn(ee_acc, __fmul_rn(src[d * EP], src[d * EP]));
    if (dc == ND - 1) ees[(ct & 1) * VQ_CODES + tid] = ee_acc;
  };

  f32x2 acc[RPL][4];               // [row i][code pair jp]: codes 8lc + 2jp, 8lc + 2jp + 1
#pragma unroll
  for (int i = 0; i < RPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x2{0.f, 0.f};
  float best[RPL];
  int bestk[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    best[i] = __builtin_huge_valf();
    bestk[i] = 0x7fffffff;
  }

  load(0);
  store(0);
  __syncthreads();
  float zz[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) zz[i] = zzs[lr + 8 * i];

  for (int st = 0; st < nsteps; ++st) {
    if (st + 1 < nsteps) load(st + 1);
    norms(st);
    const int ct = st / ND, dc = st - ct * ND;
    const float* eb = es + (st & 1) * L::E + w * 64 + 8 * lc;
    const float* zb = zs + lr * ZP + dc * VQ_DC;
#pragma unroll 1
    for (int q = 0; q < VQ_DC / 4; ++q) {   // not unrolled: hoisted operand reads of four steps would spill
      float4 zv[RPL];
#pragma unroll
      for (int i = 0; i < RPL; ++i) zv[i] = *reinterpret_cast<const float4*>(zb + 8 * i * ZP + 4 * q);
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {
        const float4 e0 = *reinterpret_cast<const float4*>(eb + (4 * q + dd) * EP);
        const float4 e1 = *reinterpret_cast<const float4*>(eb + (4 * q + dd) * EP + 4);
        const f32x2 ep[4] = {f32x2{e0.x, e0.y}, f32x2{e0.z, e0.w}, f32x2{e1.x, e1.y}, f32x2{e1.z, e1.w}};
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
          const float zi = dd == 0 ? zv[i].x : dd == 1 ? zv[i].y : dd == 2 ? zv[i].z : zv[i].w;
          const f32x2 zp = f32x2{zi, zi};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_elementwise_fma(zp, ep[j], acc[i][j]);
        }
      }
    }
    if (st + 1 < nsteps) store(st + 1);
    __syncthreads();
    if (dc == ND - 1) {   // the tile's dot products are complete (and its norms published): distances, argmin
      const float* eet = ees + (ct & 1) * VQ_CODES + w * 64 + 8 * lc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gk = ct * VQ_CODES + w * 64 + 8 * lc + j;
        const float e2 = eet[j];
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
          const float dot = (j & 1) ? acc[i][j >> 1].y : acc[i][j >> 1].x;
          const float dist = __fsub_rn(__fadd_rn(zz[i], e2), __fmul_rn(2.f, dot));
          lex_take(dist, gk, gk < K, best[i], bestk[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < RPL; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x2{0.f, 0.f};
    }
  }

  vq_finish<D, RPL>(best, bestk, es, 2 * L::E - 16 * ROWS, zs, reinterpret_cast<double*>(ees), E, N, K, row0, zq,
                    idx, counts, sqerr, zq2, zq2_bf16);
}

// Codebook-pinned form (K <= 512, D <= 64: the configs[1] codebook, 512 x 64 fp32 = 128 KB): ONE workgroup per CU
// of 64 rows stages the whole codebook into LDS once ([d][code], transposed on the way in, as the streaming
// kernel's chunks) beside its z tile, then runs the full embedding dim without a barrier -- no per-chunk staging,
// no load latency per chunk.  Same per-lane register blocks, same in-order fma chains, norms and (d, k) argmin as
// vq_fwd_kernel, so the same bits.
template <int D>
__global__ __launch_bounds__(VQ_THREADS, 1) void vq_fwd_pinned_kernel(const float* __restrict__ z,
                                                                     const float* __restrict__ E, int64_t N, int K,
                                                                     float* __restrict__ zq, int64_t* __restrict__ idx,
                                                                     float* __restrict__ counts,
                                                                     double* __restrict__ sqerr, void* __restrict__ zq2,
                                                                     int zq2_bf16) {
  constexpr int RPL = 8, ROWS = 64, ZP = D + 4, EP = VQ_CODES + 4, NQ = D / 4;
  constexpr int ZF = ROWS * ZP, EF = D * EP;
  static_assert(D % 16 == 0 && D <= 64, "pinned codebook: D 16..64");
  __shared__ __attribute__((aligned(16))) float smem[ZF + EF + VQ_CODES + ROWS];
  float* zs = smem;
  float* es = smem + ZF;                   // [D][VQ_CODES (+4)]
  float* ees = es + EF;                    // [VQ_CODES]
  float* zzs = ees + VQ_CODES;             // [ROWS]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane >> 3, lc = lane & 7;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;

  // ---- the codebook: float4 (u, dc) of thread t = quad t & 3 of dims 16 dc .. of code 128 u + (t >> 2), all in
  //      flight at once (codes >= K read as zero), then stored transposed; the z tile behind them
  float4 pre[4][D / 16];
#pragma unroll
  for (int dc = 0; dc < D / 16; ++dc)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int code = 128 * u + (tid >> 2);
      pre[u][dc] = code < K ? reinterpret_cast<const float4*>(E + (int64_t)code * D + dc * 16)[tid & 3]
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  for (int i = tid; i < ROWS * NQ; i += VQ_THREADS) {
    const int r = i / NQ, q = i - r * NQ;
    const int64_t gr = row0 + r;
    const float4 v = gr < N ? reinterpret_cast<const float4*>(z + gr * D)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(zs + r * ZP + 4 * q) = v;
  }
#pragma unroll
  for (int dc = 0; dc < D / 16; ++dc)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float* dst = es + (16 * dc + 4 * (tid & 3)) * EP + 128 * u + (tid >> 2);
      dst[0 * EP] = pre[u][dc].x;
      dst[1 * EP] = pre[u][dc].y;
      dst[2 * EP] = pre[u][dc].z;
      dst[3 * EP] = pre[u][dc].w;
    }
  __syncthreads();
  // ---- |z|^2 per row and |e_k|^2 per code: in-order sums of squares
  if (tid < ROWS) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = __fadd_rn(s, __fmul_rn(zs[tid * ZP + d], zs[tid * ZP + d]));
    zzs[tid] = s;
  }
  {
    float s = 0.f;
#pragma unroll 16
    for (int d = 0; d < D; ++d) s = __fadd_rn(s, __fmul_rn(es[d * EP + tid], es[d * EP + tid]));
    ees[tid] = s;
  }
  __syncthreads();

  f32x2 acc[RPL][4];               // [row i][code pair jp]: codes 8lc + 2jp, 8lc + 2jp + 1
#pragma unroll
  for (int i = 0; i < RPL; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x2{0.f, 0.f};
  // software-pipelined LDS reads: the z quads of step q + 1 and the code values of the next embedding index are in
  // flight while the current index's 32 packed FMAs issue (read at their use, the waves waited on LDS half the time)
  const float* eb = es + w * 64 + 8 * lc;
  const float* zb = zs + lr * ZP;
  float4 zc[RPL], zn[RPL];
#pragma unroll
  for (int i = 0; i < RPL; ++i) zc[i] = *reinterpret_cast<const float4*>(zb + 8 * i * ZP);
  float4 e0 = *reinterpret_cast<const float4*>(eb), e1 = *reinterpret_cast<const float4*>(eb + 4);
#pragma unroll 1
  for (int q = 0; q < NQ; ++q) {
    const int qn = q + 1 < NQ ? q + 1 : q;   // the last step re-reads its own quads (unused)
#pragma unroll
    for (int dd = 0; dd < 4; ++dd) {
      const int dn = 4 * q + dd + 1 < D ? 4 * q + dd + 1 : 4 * q + dd;
      const float4 n0 = *reinterpret_cast<const float4*>(eb + dn * EP);
      const float4 n1 = *reinterpret_cast<const float4*>(eb + dn * EP + 4);
      if (dd == 0) {
        // issued behind the next code values: LDS reads retire in order, so the code values' waits do not wait
        // for these
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < RPL; ++i) zn[i] = *reinterpret_cast<const float4*>(zb + 8 * i * ZP + 4 * qn);
        __builtin_amdgcn_sched_barrier(0);
      }
      const f32x2 ep[4] = {f32x2{e0.x, e0.y}, f32x2{e0.z, e0.w}, f32x2{e1.x, e1.y}, f32x2{e1.z, e1.w}};
#pragma unroll
      for (int i = 0; i < RPL; ++i) {
        const float zi = dd == 0 ? zc[i].x : dd == 1 ? zc[i].y : dd == 2 ? zc[i].z : zc[i].w;
        const f32x2 zp = f32x2{zi, zi};
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_elementwise_fma(zp, ep[j], acc[i][j]);
      }
      e0 = n0;
      e1 = n1;
    }
#pragma unroll
    for (int i = 0; i < RPL; ++i) zc[i] = zn[i];
  }
  // ---- distances and this lane's (d, k) minimum
  float best[RPL];
  int bestk[RPL];
  const float* eet = ees + w * 64 + 8 * lc;
#pragma unroll
  for (int i = 0; i < RPL; ++i) {
    best[i] = __builtin_huge_valf();
    bestk[i] = 0x7fffffff;
    const float zz = zzs[lr + 8 * i];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gk = w * 64 + 8 * lc + j;
      const float dot = (j & 1) ? acc[i][j >> 1].y : acc[i][j >> 1].x;
      const float dist = __fsub_rn(__fadd_rn(zz, eet[j]), __fmul_rn(2.f, dot));
      lex_take(dist, gk, gk < K, best[i], bestk[i]);
    }
  }
  __syncthreads();   // every wave's codebook reads are done: the E area becomes the exchange scratch
  vq_finish<D, RPL>(best, bestk, es, EF - 16 * ROWS, zs, reinterpret_cast<double*>(ees), E, N, K, row0, zq, idx,
                    counts, sqerr, zq2, zq2_bf16);
}

__global__ void vq_finalize_kernel(const float* counts, const double* sqerr, int64_t N, int K, int D, float beta,
                                   float* loss, float* perp) {
  __shared__ float part[256];
  const float invN = 1.0f / (float)N;
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float p = counts[k] * invN;
    s += p * logf(p + 1e-10f);
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float m = (float)(sqerr[0] / ((double)N * (double)D));
    loss[0] = m + beta * m;
    perp[0] = expf(-part[0]);
  }
}

__global__ void vq_bwd_kernel(const float* __restrict__ z, const float* __restrict__ E, const int64_t* __restrict__ idx,
                              const float* __restrict__ g_zq, const float* __restrict__ g_loss, int64_t N, int D,
                              float beta, float* __restrict__ dz, float* __restrict__ dE,
                              void* __restrict__ dz2, int dz2_bf16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int64_t r = i / D;
  const int d = (int)(i - r * D);
  const int64_t k = idx[r];
  const float g = g_loss ? g_loss[0] : 0.f;
  const float scale = 2.0f / (float)((double)N * (double)D);
  const float diff = E[k * D + d] - z[i];  // z_q - z
  const float v = (g_zq ? g_zq[i] : 0.f) - g * scale * diff;
  dz[i] = v;
  if (dz2) {   // operand copy for the SepCNN backward GEMMs
    if (dz2_bf16) reinterpret_cast<bf16*>(dz2)[i] = (bf16)v;
    else reinterpret_cast<float*>(dz2)[i] = v;
  }
  if (g != 0.f) atomicAdd(dE + k * D + d, g * beta * scale * diff);
}

__global__ void vq_onehot_kernel(const int64_t* idx, int64_t N, int K, float* onehot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * (int64_t)K) return;
  const int64_t r = i / K;
  onehot[i] = (idx[r] == (i - r * K)) ? 1.f : 0.f;
}

__global__ void vq_gather_kernel(const float* E, const int64_t* idx, int64_t N, int D, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int64_t r = i / D;
  out[i] = E[idx[r] * D + (i - r * D)];
}

}  // namespace


extern "C" int aw_vq_forward_ex(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx,
                                float* counts, double* sqerr, void* zq_copy, int copy_dtype, void* stream) {
  AW_REQUIRE(z && E && zq && idx && counts && sqerr, "aw_vq_forward: null pointer");
  AW_REQUIRE(!zq_copy || ((copy_dtype == AW_BF16 || copy_dtype == AW_F32) && ((uintptr_t)zq_copy % 16) == 0),
             "aw_vq_forward_ex: zq_copy must be 16-B aligned bf16 or f32");
  const int cbf = copy_dtype == AW_BF16;
  AW_REQUIRE(N >= 0 && K > 0, "aw_vq_forward: bad N/K");
  AW_REQUIRE(((uintptr_t)z % 16) == 0 && ((uintptr_t)E % 16) == 0 && ((uintptr_t)zq % 16) == 0,
             "aw_vq_forward: z/E/zq must be 16-B aligned");
  if (N == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 64-row workgroups while they fill every CU twice; 32-row ones below that, where two of them fit one CU's LDS
  // (D <= 64: 78 KB each) -- the bench shape N 16384 then runs 512 workgroups, two per CU
  static int rows_env = -1;
  if (rows_env < 0) {
    const char* e = getenv("ARCWELD_VQ_ROWS");
    rows_env = e ? atoi(e) : 0;
  }
  const bool half = rows_env ? rows_env == 32 : (N < 512 * 64 && D <= 64);
  const dim3 grid(aw_cdiv(N, half ? 32 : 64));
  // the codebook-pinned form whenever the codebook fits beside a 64-row z tile (ARCWELD_VQ_ROWS=32 / 64 pins the
  // streaming kernel for A/B runs)
  if (!rows_env && K <= VQ_CODES && (D == 16 || D == 32 || D == 64)) {
    const dim3 g64(aw_cdiv(N, 64));
    if (D == 16) hipLaunchKernelGGL((vq_fwd_pinned_kernel<16>), g64, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts,
                                    sqerr, zq_copy, cbf);
    else if (D == 32) hipLaunchKernelGGL((vq_fwd_pinned_kernel<32>), g64, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx,
                                         counts, sqerr, zq_copy, cbf);
    else hipLaunchKernelGGL((vq_fwd_pinned_kernel<64>), g64, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr,
                            zq_copy, cbf);
    return aw::check_launch("aw_vq_forward");
  }
#define AW_VQ_CASE(DD)                                                                                               \
  case DD:                                                                                                           \
    if (half) hipLaunchKernelGGL((vq_fwd_kernel<DD, 4>), grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr, \
                                 zq_copy, cbf);                                                                      \
    else hipLaunchKernelGGL((vq_fwd_kernel<DD, 8>), grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr,     \
                            zq_copy, cbf);                                                                           \
    break;
  switch (D) {
    AW_VQ_CASE(16)
    AW_VQ_CASE(32)
    AW_VQ_CASE(64)
    AW_VQ_CASE(128)
    AW_VQ_CASE(256)
    default: aw::set_error("aw_vq_forward: unsupported embedding dim %d (16/32/64/128/256)", D); return AW_ERR_ARG;
  }
#undef AW_VQ_CASE
  return aw::check_launch("aw_vq_forward");
}

extern "C" int aw_vq_forward(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx,
                             float* counts, double* sqerr, void* stream) {
  return aw_vq_forward_ex(z, E, N, K, D, zq, idx, counts, sqerr, nullptr, AW_F32, stream);
}

extern "C" int aw_vq_finalize(const float* counts, const double* sqerr, int64_t N, int K, int D, float beta,
                              float* loss, float* perplexity, void* stream) {
  AW_REQUIRE(counts && sqerr && loss && perplexity && N > 0 && K > 0 && D > 0, "aw_vq_finalize: bad args");
  hipLaunchKernelGGL(vq_finalize_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), counts, sqerr,
                     N, K, D, beta, loss, perplexity);
  return aw::check_launch("aw_vq_finalize");
}

extern "C" int aw_vq_backward_ex(const float* z, const float* E, const int64_t* idx, const float* g_zq,
                                 const float* g_loss, int64_t N, int K, int D, float beta, float* dz, float* dE,
                                 void* dz_copy, int copy_dtype, void* stream) {
  AW_REQUIRE(z && E && idx && dz && dE && N >= 0 && K > 0 && D > 0, "aw_vq_backward: bad args");
  AW_REQUIRE(!dz_copy || copy_dtype == AW_BF16 || copy_dtype == AW_F32, "aw_vq_backward_ex: bad copy dtype");
  if (N == 0) return AW_OK;
  const int64_t n = N * D;
  hipLaunchKernelGGL(vq_bwd_kernel, dim3(aw_cdiv(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), z,
                     E, idx, g_zq, g_loss, N, D, beta, dz, dE, dz_copy, copy_dtype == AW_BF16 ? 1 : 0);
  return aw::check_launch("aw_vq_backward");
}

extern "C" int aw_vq_backward(const float* z, const float* E, const int64_t* idx, const float* g_zq,
                              const float* g_loss, int64_t N, int K, int D, float beta, float* dz, float* dE,
                              void* stream) {
  return aw_vq_backward_ex(z, E, idx, g_zq, g_loss, N, K, D, beta, dz, dE, nullptr, AW_F32, stream);
}

extern "C" int aw_vq_onehot(const int64_t* idx, int64_t N, int K, float* onehot, void* stream) {
  AW_REQUIRE(idx && onehot && N >= 0 && K > 0, "aw_vq_onehot: bad args");
  if (N == 0) return AW_OK;
  const int64_t n = N * (int64_t)K;
  hipLaunchKernelGGL(vq_onehot_kernel, dim3(aw_cdiv(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), idx,
                     N, K, onehot);
  return aw::check_launch("aw_vq_onehot");
}

extern "C" int aw_vq_gather(const float* E, const int64_t* idx, int64_t N, int D, float* out, void* stream) {
  AW_REQUIRE(E && idx && out && N >= 0 && D > 0, "aw_vq_gather: bad args");
  if (N == 0) return AW_OK;
  const int64_t n = N * D;
  hipLaunchKernelGGL(vq_gather_kernel, dim3(aw_cdiv(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), E,
                     idx, N, D, out);
  return aw::check_launch("aw_vq_gather");
}
