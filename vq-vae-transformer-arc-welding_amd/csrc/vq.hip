// Vector quantizer (model/vector_quantizer.py:59-131) for gfx950.
//
// Forward: distances follow the reference expression exactly in fp32:
//     d_k = fl( fl(|z|^2 + |e_k|^2) - 2 * dot(z, e_k) ),  dot = k-ordered fmaf chain over the embedding dim
// (torch's CPU sgemm on this shape is bit-identical to that chain -- measured), so the
// argmin (lexicographic (d, k) minimum == torch.argmin first-index tie rule) is bit-exact.  Two kernels:
//   * vq_fwd_pinned_kernel (K <= 512, D <= 64, the configs[1] codebook): the codebook pinned in LDS, the dot
//     products on the f32-input MFMA, which is bit for bit the same fmaf chain;
//   * vq_fwd_kernel (any K, D <= 256): register-blocked fp32 VALU tiles with the codebook streamed through LDS.
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
  // counts: this workgroup's partial histogram (the caller offsets it by blockIdx % count_groups)
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
                                                               float* __restrict__ counts, int cgroups,
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
                    idx, counts + (int64_t)(blockIdx.x % cgroups) * K, sqerr, zq2, zq2_bf16);
}

// Codebook-pinned form (K <= 512, D <= 64: the configs[1] codebook, 512 x 64 fp32 = 128 KB): ONE workgroup per CU
// of 64 rows keeps the whole codebook in LDS and runs the dot products on the f32-input MFMA
// (v_mfma_f32_32x32x2_f32).  That instruction is bit for bit a k-ordered fmaf chain -- D = fma(a_k1, b_k1,
// fma(a_k0, b_k0, C)) with one rounding per product (cdna_hip_programming.md, 'FP32-input MFMA') -- so step s over
// dims (2s, 2s + 1) continues exactly the chain the VALU kernel runs, at the vector rate but off the vector pipe,
// with four steps' operands per 16-B LDS read.  Wave w owns codes 64w .. 64w + 63 (M, two 32-code tiles) x all 64
// rows (N, two 32-row tiles); lane l ends with row (l & 31) of each row tile against 32 of the wave's codes.
//
// The codebook arrives in 16-dim chunks: all of its loads are issued at once, and each chunk is stored and its MFMA
// steps run as soon as its data is in (one LDS barrier per chunk), so the load latency overlaps the matrix work;
// the norms |e_k|^2 and |z|^2 accumulate chunk by chunk beside the MFMAs.  The codebook stays in LDS to the end:
// the epilogue gathers z_q's code rows from it (no dependent global load).
template <int D> struct VqPinLds {
  static constexpr int ROWS = 64;
  static constexpr int ES = 0, ZS = ES + VQ_CODES * D, EES = ZS + ROWS * D, ZZS = EES + VQ_CODES;
  static constexpr int RD = ZZS + ROWS, HIST = RD + 2 * ROWS, RED = HIST + VQ_CODES;   // RD: ROWS u64 keys
  static constexpr int TOTAL = RED + 16;                     // floats (RED: 8 doubles)
  static_assert(TOTAL * 4 <= 160 * 1024, "pinned VQ LDS");
};

// Float offset of permuted position p of row c in a [c][D] image.  Positions: dim d sits at (d & 1) * D/2 + (d >> 1)
// (even dims, then odd), so MFMA lane half h reads steps s .. s + 3 (dims 2s + h, ...) as one float4 at h * D/2 + s;
// 16-B quads are XOR-swizzled by the row, so the 16 lanes of a ds_read_b128 group (rows distinct mod 16) hit 16
// distinct quads = all 64 banks (for D = 64; 2- / 4-way at D = 32 / 16).
template <int D> __device__ __forceinline__ int vq_pos(int c, int p) {
  return c * D + ((((p >> 2) ^ c) & (D / 4 - 1)) << 2) + (p & 3);
}

// Wave sum of a double on the VALU only (no LDS round trips): DPP within 16-lane rows (quad swaps, half-row and row
// mirrors), then gfx950's v_permlane16_swap / v_permlane32_swap for lanes 16 and 32 apart.  Every lane ends with the
// total (each step adds the same two values on both partners).
template <int CTRL> __device__ __forceinline__ double vq_dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ double vq_wave_sum_d(double v) {
  v += vq_dpp_d<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  v += vq_dpp_d<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  v += vq_dpp_d<0x141>(v);   // row_half_mirror
  v += vq_dpp_d<0x140>(v);   // row_mirror
  const int lane = __lane_id();
  {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    const bool odd = (lane >> 4) & 1;   // rows 1, 3 received rows 0, 2 in [0]; rows 0, 2 received rows 1, 3 in [1]
    const uint32_t plo = odd ? lo[0] : lo[1], phi = odd ? hi[0] : hi[1];
    v += __longlong_as_double((long long)(((uint64_t)phi << 32) | plo));
  }
  {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    const bool up = lane >= 32;
    const uint32_t plo = up ? lo[0] : lo[1], phi = up ? hi[0] : hi[1];
    v += __longlong_as_double((long long)(((uint64_t)phi << 32) | plo));
  }
  return v;
}

__device__ __forceinline__ void vq_lds_barrier() {   // LDS-only: no wait for the global loads still in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int D>
__global__ __launch_bounds__(VQ_THREADS, 1) void vq_fwd_pinned_kernel(const float* __restrict__ z,
                                                                     const float* __restrict__ E, int64_t N, int K,
                                                                     float* __restrict__ zq, int64_t* __restrict__ idx,
                                                                     float* __restrict__ counts, int cgroups,
                                                                     double* __restrict__ sqerr, void* __restrict__ zq2,
                                                                     int zq2_bf16) {
  typedef __attribute__((ext_vector_type(16))) float f32x16;
  using L = VqPinLds<D>;
  constexpr int ROWS = L::ROWS, NQ = D / 4, NCH = D / 16, H2 = D / 2;
  constexpr int ZPT = (ROWS * NQ + VQ_THREADS - 1) / VQ_THREADS;   // z float4 per thread
  static_assert(D % 16 == 0 && D <= 64, "pinned codebook: D 16..64");
  __shared__ __attribute__((aligned(16))) float smem[L::TOTAL];
  float* es = smem + L::ES;                // [VQ_CODES][D] permuted + swizzled (vq_pos)
  float* zs = smem + L::ZS;                // [ROWS][D] likewise
  float* ees = smem + L::EES;              // [VQ_CODES]: |e_k|^2, NaN for k >= K
  float* zzs = smem + L::ZZS;              // [ROWS]
  // [ROWS] lexicographic (d, k) row minima as 64-bit keys (order-preserving d bits above k), merged by LDS atomic min
  unsigned long long* rkey = reinterpret_cast<unsigned long long*>(smem + L::RD);
  float* hist = smem + L::HIST;            // [VQ_CODES] this workgroup's code counts
  double* red = reinterpret_cast<double*>(smem + L::RED);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, jr = lane & 31;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;

  // ---- loads: the z tile first, then the codebook chunk by chunk (float4 (dc, u) of thread t = quad t & 3 of dims
  //      16 dc .. of code 128 u + (t >> 2)), all in flight at once.  Addresses are clamped instead of predicated:
  //      codes >= K hold a copy of code K - 1 and are excluded by their NaN norm, rows >= N a copy of row N - 1 and
  //      are never written.
  float4 zr[ZPT];
#pragma unroll
  for (int i = 0; i < ZPT; ++i) {
    const int it = tid + i * VQ_THREADS, r = it / NQ, q = it - r * NQ;
    const int64_t gr = min(row0 + r, N - 1);
    if (it < ROWS * NQ) zr[i] = reinterpret_cast<const float4*>(z + gr * D)[q];
  }
  float4 pe[NCH][4];
#pragma unroll
  for (int dc = 0; dc < NCH; ++dc)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int code = min(128 * u + (tid >> 2), K - 1);
      pe[dc][u] = reinterpret_cast<const float4*>(E + (int64_t)code * D + dc * 16)[tid & 3];
      if (u == 3) __builtin_amdgcn_sched_barrier(0);   // issue in chunk order: chunk dc waits only for its own
    }
  // a float4 of dims 4q .. 4q + 3 goes to the image as two 8-B halves: (4q, 4q + 2) at 2q, (4q + 1, 4q + 3) at D/2 + 2q
  auto put4 = [&](float* img, int c, int q, const float4& v) {
    *reinterpret_cast<float2*>(img + vq_pos<D>(c, 2 * q)) = make_float2(v.x, v.z);
    *reinterpret_cast<float2*>(img + vq_pos<D>(c, H2 + 2 * q)) = make_float2(v.y, v.w);
  };
#pragma unroll
  for (int i = 0; i < ZPT; ++i) {
    const int it = tid + i * VQ_THREADS, r = it / NQ, q = it - r * NQ;
    if (it < ROWS * NQ) put4(zs, r, q, zr[i]);
  }
  hist[tid] = 0.f;
  if (tid < ROWS) rkey[tid] = ~0ull;

  // ---- chunk loop: per 16-dim chunk, 8 MFMA steps (two groups of four) and the norms' next 16 terms
  f32x16 acc[2][2];                // [code tile mi][row tile ni]
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  // in-order fmaf chains of squares (s = fma(x_d, x_d, s), d = 0, 1, ...: the kernels' norms since round 1):
  // |e_k|^2 of code tid and |z|^2 of row lane (every wave computes the rows' sums; wave 7 publishes them).  A chunk's
  // 16 values are read with the chunk's first operands; the two 16-long dependent chains then run one link per MFMA
  // pair inside the chunk's MFMA groups (issued as their own block they stalled the wave's issue -- and with it its
  // next MFMAs -- for ~400 cycles per chunk)
  float ee = 0.f, zz = 0.f;
  auto ld16 = [&](const float* img, int c, int dc, float (&v)[16]) {   // dims 16 dc .. 16 dc + 15, in dim order
    const float4 e0 = *reinterpret_cast<const float4*>(img + vq_pos<D>(c, 8 * dc));
    const float4 e1 = *reinterpret_cast<const float4*>(img + vq_pos<D>(c, 8 * dc + 4));
    const float4 o0 = *reinterpret_cast<const float4*>(img + vq_pos<D>(c, H2 + 8 * dc));
    const float4 o1 = *reinterpret_cast<const float4*>(img + vq_pos<D>(c, H2 + 8 * dc + 4));
    const float ev[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
    const float ov[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[2 * i] = ev[i];
      v[2 * i + 1] = ov[i];
    }
  };
  const int ca = 64 * w + jr;      // this lane's A row (code) in tile mi: ca + 32 mi; B row (z row): jr + 32 ni
  auto ops = [&](int dc, int g, float4 (&a)[2], float4 (&b)[2]) {   // steps 8 dc + 4 g .. + 3 of lane half h
    const int p = h * H2 + 8 * dc + 4 * g;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a[t] = *reinterpret_cast<const float4*>(es + vq_pos<D>(ca + 32 * t, p));
      b[t] = *reinterpret_cast<const float4*>(zs + vq_pos<D>(jr + 32 * t, p));
    }
  };
  // 16 MFMAs (four steps x 2 x 2 tiles), add i of each norm chain after MFMA 2i + 1
  auto mma4 = [&](const float4 (&a)[2], const float4 (&b)[2], const float* se, const float* sz) {
    const float av[2][4] = {{a[0].x, a[0].y, a[0].z, a[0].w}, {a[1].x, a[1].y, a[1].z, a[1].w}};
    const float bv[2][4] = {{b[0].x, b[0].y, b[0].z, b[0].w}, {b[1].x, b[1].y, b[1].z, b[1].w}};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi][s4], bv[ni][s4], acc[mi][ni], 0, 0, 0);
        ee = __builtin_fmaf(se[2 * s4 + mi], se[2 * s4 + mi], ee);
        zz = __builtin_fmaf(sz[2 * s4 + mi], sz[2 * s4 + mi], zz);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // the two MFMAs,
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // then the two adds
      }
  };
  // chunk dc + 1 is stored while chunk dc computes (after its first MFMA group), and its barrier sits between chunk
  // dc's two MFMA groups, so the first operands of chunk dc + 1 are read before the second group issues: the matrix
  // pipe does not wait on LDS latency at a chunk boundary
#pragma unroll
  for (int u = 0; u < 4; ++u) put4(es, 128 * u + (tid >> 2), tid & 3, pe[0][u]);
  vq_lds_barrier();
  float4 a0[2], b0[2], a1[2], b1[2];
  float ev[16], zv[16];
  ops(0, 0, a0, b0);
  ld16(es, tid, 0, ev);
  ld16(zs, lane, 0, zv);
#pragma unroll
  for (int dc = 0; dc < NCH; ++dc) {
    ops(dc, 1, a1, b1);
    float se[16], sz[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      se[i] = ev[i];
      sz[i] = zv[i];
    }
    mma4(a0, b0, se, sz);
    if (dc + 1 < NCH) {   // behind the first MFMA group: the chunk's loads get that much longer to land
#pragma unroll
      for (int u = 0; u < 4; ++u) put4(es, 128 * u + (tid >> 2), 4 * (dc + 1) + (tid & 3), pe[dc + 1][u]);
      vq_lds_barrier();
      ops(dc + 1, 0, a0, b0);
      ld16(es, tid, dc + 1, ev);
      ld16(zs, lane, dc + 1, zv);
      __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs below
    }
    mma4(a1, b1, se + 8, sz + 8);
  }
  ees[tid] = tid < K ? ee : __builtin_nanf("");
  if (w == 7) zzs[lane] = zz;
  vq_lds_barrier();

  // ---- distances d = fl(fl(|z|^2 + |e|^2) - 2 dot) as fma(-2, dot, s) (2 dot is exact, so the one rounding is the
  //      reference's), two codes per packed op; this lane's minimum per row over its 32 codes, visited in ascending
  //      k (accumulator register r of tile mi holds code 64w + 32mi + 8(r >> 2) + 4h + (r & 3)), so a strict <
  //      keeps the first index of a tie.  NaN distances (codes >= K, NaN inputs) never compare less; a lane left
  //      with none reports (+inf, its first code), which the lexicographic merge below ranks behind every finite
  //      candidate.
  //      The two rows run interleaved (independent compare chains), and the running index is the register
  //      position j = 16 mi + 4 g + r, a literal in each select, mapped to its code once at the end.
  float best[2] = {__builtin_huge_valf(), __builtin_huge_valf()};
  int bj[2] = {0, 0};
  {
    const float zrow[2] = {zzs[jr], zzs[jr + 32]};
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 e4 = *reinterpret_cast<const float4*>(ees + 64 * w + 32 * mi + 8 * g + 4 * h);
        float dv[2][4];
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const f32x2 s01 = f32x2{zrow[ni], zrow[ni]} + f32x2{e4.x, e4.y};
          const f32x2 s23 = f32x2{zrow[ni], zrow[ni]} + f32x2{e4.z, e4.w};
          const f32x2 d01 = __builtin_elementwise_fma(
              f32x2{-2.f, -2.f}, f32x2{acc[mi][ni][4 * g], acc[mi][ni][4 * g + 1]}, s01);
          const f32x2 d23 = __builtin_elementwise_fma(
              f32x2{-2.f, -2.f}, f32x2{acc[mi][ni][4 * g + 2], acc[mi][ni][4 * g + 3]}, s23);
          dv[ni][0] = d01.x, dv[ni][1] = d01.y, dv[ni][2] = d23.x, dv[ni][3] = d23.y;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            // the running minimum as v_min (off the compare's VCC: the next compare does not wait for a select);
            // v_min never takes a NaN over a number, as the strict < never does
            const bool t = dv[ni][r] < best[ni];
            best[ni] = __builtin_fminf(best[ni], dv[ni][r]);
            bj[ni] = t ? 16 * mi + 4 * g + r : bj[ni];
          }
      }
  }
  int bestk[2];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) bestk[ni] = 64 * w + 4 * h + 2 * bj[ni] - (bj[ni] & 3);   // = 32 mi + 8 g + r
  // ---- lexicographic (d, k) merge across the 16 lane candidates of a row (2 lane halves x 8 waves): one LDS 64-bit
  //      atomic min per lane and row on the key (sortable d << 32 | k).  The float -> sortable map (sign set: all
  //      bits flipped, else the sign bit set) orders the keys as the floats; the candidates are never NaN (a lane
  //      without a finite distance reports +inf), and -0 cannot occur (a distance is an exact zero only as x - x).
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const uint32_t b = __float_as_uint(best[ni]);
    const uint32_t u = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    atomicMin(rkey + jr + 32 * ni, ((unsigned long long)u << 32) | (uint32_t)bestk[ni]);
  }
  vq_lds_barrier();
  // ---- thread (row r, quad q) reads its row's winner (one LDS broadcast read of the key), takes e_k's quad from
  //      the pinned codebook and writes z_q (+ the operand copy) coalesced; the q == 0 thread of a row writes idx and
  //      counts the code in LDS.  The items of a thread are unrolled and only their stores predicated, so their LDS
  //      chains overlap.
  double se = 0.0;
  constexpr int IPT = (ROWS * NQ + VQ_THREADS - 1) / VQ_THREADS;
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int it = min(tid + i * VQ_THREADS, ROWS * NQ - 1);
    const int r = it / NQ, q = it - r * NQ;
    const int64_t row = row0 + r;
    const bool live = tid + i * VQ_THREADS < ROWS * NQ && row < N;
    int bk = (int)(uint32_t)rkey[r];
    if (bk < 0 || bk >= K) bk = 0;  // all-NaN row guard (torch would return the NaN position)
    if (live && q == 0) {
      idx[row] = bk;
      atomicAdd(hist + bk, 1.0f);
    }
    const float2 e02 = *reinterpret_cast<const float2*>(es + vq_pos<D>(bk, 2 * q));
    const float2 e13 = *reinterpret_cast<const float2*>(es + vq_pos<D>(bk, H2 + 2 * q));
    const float2 z02 = *reinterpret_cast<const float2*>(zs + vq_pos<D>(r, 2 * q));
    const float2 z13 = *reinterpret_cast<const float2*>(zs + vq_pos<D>(r, H2 + 2 * q));
    const float d0 = __fsub_rn(e02.x, z02.x), d1 = __fsub_rn(e13.x, z13.x);
    const float d2 = __fsub_rn(e02.y, z02.y), d3 = __fsub_rn(e13.y, z13.y);
    float4 o;
    o.x = __fadd_rn(z02.x, d0);  // z + (z_q - z).detach()
    o.y = __fadd_rn(z13.x, d1);
    o.z = __fadd_rn(z02.y, d2);
    o.w = __fadd_rn(z13.y, d3);
    if (live) {
      // write-through stores: the lines leave L2 now instead of at the end-of-kernel release
      aw_st_wt(zq + row * D + 4 * q, f32x4{o.x, o.y, o.z, o.w});
      if (zq2) {   // the GEMM operand copy of z_q (the decoder's first conv reads it): no separate cast launch
        if (zq2_bf16) {
          typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
          const bf16x4 v = bf16x4{(bf16)o.x, (bf16)o.y, (bf16)o.z, (bf16)o.w};
          aw_st_wt(reinterpret_cast<bf16x4*>(zq2) + row * NQ + q, __builtin_bit_cast(u32x2, v));
        } else {
          aw_st_wt(reinterpret_cast<float4*>(zq2) + row * NQ + q, f32x4{o.x, o.y, o.z, o.w});
        }
      }
      se += (double)(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
    }
  }
  se = vq_wave_sum_d(se);
  if (lane == 0) red[w] = se;
  vq_lds_barrier();   // LDS only: no wait for this workgroup's z_q stores
  // the histogram goes to partial blockIdx % cgroups: the adds into one address stay cgroups times fewer (every
  // workgroup adding into the same 2 KB serialises at the memory-side atomic units: 2.5 us of drain at cgroups 1)
  if (tid < K) {
    const float c = hist[tid];
    if (c != 0.f) atomicAdd(counts + (int64_t)(blockIdx.x % cgroups) * K + tid, c);
  }
  if (tid == 0) {
    double t = 0.0;
#pragma unroll
    for (int v = 0; v < 8; ++v) t += red[v];
    atomicAdd(sqerr, t);
  }
}

__global__ void vq_finalize_kernel(const float* counts, int cgroups, const double* sqerr, int64_t N, int K, int D,
                                   float beta, float* loss, float* perp) {
  __shared__ float part[256];
  const float invN = 1.0f / (float)N;
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    float c = counts[k];
    for (int g = 1; g < cgroups; ++g) c += counts[(int64_t)g * K + k];   // integer-valued: exact in any order
    const float p = c * invN;
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


extern "C" int aw_vq_forward_ex2(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx,
                                 float* counts, int count_groups, double* sqerr, void* zq_copy, int copy_dtype,
                                 void* stream) {
  AW_REQUIRE(z && E && zq && idx && counts && sqerr, "aw_vq_forward: null pointer");
  AW_REQUIRE(count_groups >= 1 && count_groups <= AW_VQ_COUNT_GROUPS_MAX, "aw_vq_forward_ex2: count_groups 1..%d",
             AW_VQ_COUNT_GROUPS_MAX);
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
                                    count_groups, sqerr, zq_copy, cbf);
    else if (D == 32) hipLaunchKernelGGL((vq_fwd_pinned_kernel<32>), g64, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx,
                                         counts, count_groups, sqerr, zq_copy, cbf);
    else hipLaunchKernelGGL((vq_fwd_pinned_kernel<64>), g64, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, count_groups,
                            sqerr, zq_copy, cbf);
    return aw::check_launch("aw_vq_forward");
  }
#define AW_VQ_CASE(DD)                                                                                               \
  case DD:                                                                                                           \
    if (half) hipLaunchKernelGGL((vq_fwd_kernel<DD, 4>), grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts,   \
                                 count_groups, sqerr, zq_copy, cbf);                                                 \
    else hipLaunchKernelGGL((vq_fwd_kernel<DD, 8>), grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts,        \
                            count_groups, sqerr, zq_copy, cbf);                                                      \
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

extern "C" int aw_vq_forward_ex(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx,
                                float* counts, double* sqerr, void* zq_copy, int copy_dtype, void* stream) {
  return aw_vq_forward_ex2(z, E, N, K, D, zq, idx, counts, 1, sqerr, zq_copy, copy_dtype, stream);
}

extern "C" int aw_vq_forward(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx,
                             float* counts, double* sqerr, void* stream) {
  return aw_vq_forward_ex2(z, E, N, K, D, zq, idx, counts, 1, sqerr, nullptr, AW_F32, stream);
}

extern "C" int aw_vq_finalize_ex(const float* counts, int count_groups, const double* sqerr, int64_t N, int K, int D,
                                 float beta, float* loss, float* perplexity, void* stream) {
  AW_REQUIRE(counts && sqerr && loss && perplexity && N > 0 && K > 0 && D > 0, "aw_vq_finalize: bad args");
  AW_REQUIRE(count_groups >= 1 && count_groups <= AW_VQ_COUNT_GROUPS_MAX, "aw_vq_finalize_ex: count_groups 1..%d",
             AW_VQ_COUNT_GROUPS_MAX);
  hipLaunchKernelGGL(vq_finalize_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), counts,
                     count_groups, sqerr, N, K, D, beta, loss, perplexity);
  return aw::check_launch("aw_vq_finalize");
}

extern "C" int aw_vq_finalize(const float* counts, const double* sqerr, int64_t N, int K, int D, float beta,
                              float* loss, float* perplexity, void* stream) {
  return aw_vq_finalize_ex(counts, 1, sqerr, N, K, D, beta, loss, perplexity, stream);
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
