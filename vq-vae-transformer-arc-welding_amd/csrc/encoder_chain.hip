// Fused per-token encoder ResBlock chain (bf16 operands, fp32 accumulation) -- aw_encoder_chain_fwd.
//
// The encoder's ResBlocks act on every token alone (centre taps of k = 3 convs on length-1 slices,
// model/vq_vae_patch_embedd.py:60-74, 103-110), so a 64-token tile can run the whole stack without any other
// tile's data.  One 512-thread workgroup per tile (the whole 160 KB LDS of a CU, two waves per SIMD):
//   * the block input a = gelu(x) (bf16, 64 x 512) stays in LDS as the B operand of both GEMMs of a block;
//   * the residual x (f32) stays in registers in the MFMA accumulator layout for the whole launch;
//   * the 2R weight matrices (K-step-major copies, relayout mode 6) stream as ONE sequence of T = 32 R K-steps (512 rows x 32 k, 32 KB each) through a
//     three-buffer LDS-DMA ring that never drains: step t waits (counted vmcnt, raw s_barrier) for the step
//     issued two steps earlier, so the next matrix's first steps are in flight across every epilogue;
//   * each wave owns 64 output channels for all 64 tokens: D[n][m] = W[n][:] . a[m][:] with
//     v_mfma_f32_16x16x32_bf16 (first operand = weights, so a lane holds 4 consecutive channels of one token).
// The saved tensors of the backward (h, a1 = gelu(h), x, gelu(x) per block) are not written by the epilogues:
// every K-step of the following GEMM issues exactly two buffer stores -- one 16-x-16 register fragment (x or h)
// and one 8-B-per-lane slice of the LDS operand image it is reading (gelu(x) during conv1, a1 during conv2) --
// so 5 KB/token/block of HBM writes overlap the weight stream instead of stalling every tile at each epilogue.
// Buffer descriptors clip the ragged last tile (rows >= N are dropped by the hardware), so every step issues the
// same number of VMEM operations and the vmcnt counts are exact.
//
// LDS images (16-B chunk swizzles checked against the ds_read_b128 lane groups of MI355X_MICROARCH.md § LDS):
//   activation image [64 m][1024 B]: logical chunk c of row m at physical chunk c ^ (m & 15);
//   weight stage     [512 n][64 B]:  logical chunk c of row n at physical chunk c ^ G[(n >> 2) & 3],
//                                    G = {0, 2, 3, 1} (the 16 lanes of every read group hit 16 distinct
//                                    bank quads).
#include "common.h"

#pragma clang diagnostic ignored "-Winline-asm"

// EC_PROBE (timing probes only, tools/probe/chain_probe.py; 0 in the library): bit 1 drops the overlapped stores,
// bit 4 the MFMAs; bits 8 / 16 / 32 point the x / image-copy / h stores at an empty range (issued, no traffic);
// bit 64 loosens every step wait by 32 operations (wrong results: measures the store/DMA coupling).  EC_AUX: the
// cache policy of the stores (gfx950 aux bits: 1 sc0, 2 nt, 16 sc1); nt measured 26 % faster than the default
// policy at N 16384, R 8 (tools/probe/chain_probe.py).
#ifndef EC_PROBE
#define EC_PROBE 0
#endif

namespace {

constexpr int EC_H = 512;
constexpr int EC_ROWS = 64;
constexpr int EC_THREADS = 512;
constexpr int EC_BK = 32;                          // K per step (one 16x16x32 MFMA deep)
constexpr int EC_STEPS = EC_H / EC_BK;             // 16 per matrix
constexpr int EC_NBUF = 3;
constexpr int ACT_BYTES = EC_ROWS * EC_H * 2;      // 64 KB
constexpr int STAGE_BYTES = EC_H * EC_BK * 2;      // 32 KB
constexpr int EC_LDS = ACT_BYTES + EC_NBUF * STAGE_BYTES;   // 160 KB
constexpr int EC_DMA_PER_STEP = 4;                 // buffer_load ... lds per thread per K-step
constexpr int EC_ST_PER_STEP = 2;                  // buffer stores per thread per K-step
constexpr int EC_RSRC_FLAGS = 0x00020000;

typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef int v2i32 __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ int act_off(int m, int chunk) { return m * 1024 + ((chunk ^ (m & 15)) << 4); }
__device__ __forceinline__ int wswz(int n) { return (0x1E4 >> (2 * ((n >> 2) & 3))) & 3; }   // G = {0,2,3,1}
__device__ __forceinline__ int w_off(int n, int chunk) { return n * 64 + ((chunk ^ wswz(n)) << 4); }

__device__ __forceinline__ v4i32 make_desc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  return v4i32{(int)__builtin_amdgcn_readfirstlane((uint32_t)b),
               (int)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu),
               (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000};
}

// the rows [row0, row0 + 64) of a [N][512] output (row_bytes per row) as a range-checked buffer; a null output
// gets an empty range, so its stores are still issued (and counted) but write nothing
__device__ __forceinline__ rsrc_t tile_rsrc(const void* base, int64_t row0, int64_t N, int row_bytes, int probe = 0) {
  if (EC_PROBE & probe) base = nullptr;
  const int64_t rows = base ? (N - row0 < EC_ROWS ? N - row0 : EC_ROWS) : 0;
  char* p = base ? (char*)base + row0 * row_bytes : nullptr;
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)(rows * row_bytes), EC_RSRC_FLAGS);
}

// K-step s of a weight matrix W (K-step-major [16][512 out][32 in] bf16: every K-step one contiguous 32 KB block,
// spread over all L2 channels; the [out][in] layout read 64 B per 1 KB row and measured 6-7 % slower) into a
// stage image: chunk q = i*512 + tid (lane-linear in LDS) holds row q >> 2, physical chunk q & 3 -> logical chunk
// (q & 3) ^ G(row).  The per-lane part of the source offset does not depend on the step (4 VGPRs for the whole
// launch); the step goes in the scalar offset.
struct WeightLanes {
  int off[EC_DMA_PER_STEP];
  __device__ explicit WeightLanes(int tid) {
#pragma unroll
    for (int i = 0; i < EC_DMA_PER_STEP; ++i) {
      const int q = i * EC_THREADS + tid;
      const int n = q >> 2;
      off[i] = n * (EC_BK * 2) + (((q & 3) ^ wswz(n)) << 4);
    }
  }
};

__device__ __forceinline__ void stage_weights(const v4i32& desc, uint32_t stage_lds, const WeightLanes& L, int tid,
                                              int s) {
  const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)(tid >> 6));   // wave-uniform: the M0 base is an SGPR
  const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(s * STAGE_BYTES));
#pragma unroll
  for (int i = 0; i < EC_DMA_PER_STEP; ++i) {
    const uint32_t m0 = stage_lds + (uint32_t)(i * EC_THREADS * 16) + wv * 1024u;
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(m0), "v"(L.off[i]),
                 "s"(desc), "s"(soff)
                 : "memory", "m0");
  }
}

// ring step t of the whole launch: matrix t / 16 (W1[0], W2[0], W1[1], ...), K-step t % 16, buffer t % 3
__device__ __forceinline__ void issue_step(const aw_encoder_chain_args& P, int t, int T, uint32_t ring,
                                           const WeightLanes& L, int tid) {
  if (t >= T) return;
  const int mat = t >> 4;
  const void* W = (mat & 1) ? P.W2[mat >> 1] : P.W1[mat >> 1];
  stage_weights(make_desc(W, EC_H * EC_H * 2), ring + (uint32_t)((t % EC_NBUF) * STAGE_BYTES), L, tid, t & 15);
}

// step t may read its buffer once every wave's DMA of step t has landed: the VMEM operations issued after it are
// step t-2's stores, step t+1's DMA (absent at the last step), step t-1's stores and, for the first two steps of a
// conv2, the 16 h stores of the conv1 epilogue -- wait for all older ones, then the barrier publishes the stage (the
// same barrier retires the previous readers of the buffer step t+2 is about to overwrite).
template <int EXTRA0>
__device__ __forceinline__ void step_sync(bool more) {
  constexpr int EXTRA = EXTRA0 + ((EC_PROBE & 64) ? 32 : 0);
  static_assert(2 * EC_ST_PER_STEP + EC_DMA_PER_STEP == 8, "vmcnt counts");
  if (more)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(8 + EXTRA) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(4 + EXTRA) : "memory");
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifndef EC_AUX
#define EC_AUX 2
#endif
constexpr int EC_STORE_AUX = EC_AUX;
__device__ __forceinline__ void store_frag(rsrc_t rs, int off, const f32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, v), rs, off, 0, EC_STORE_AUX);
}
__device__ __forceinline__ void store_frag(rsrc_t rs, int off, const uint2& v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i32, v), rs, off, 0, EC_STORE_AUX);
}

// One GEMM of the chain (16 ring steps starting at t0) with its share of the overlapped stores: at K-step s the
// residual fragment xr[s / 4][s % 4] goes to `xrs` (an empty range during conv2: the store keeps the per-step count)
// and slice s of the operand image (8 B per thread, half a row per wave) goes to `irs`.  EXTRA: VMEM operations
// issued between the previous GEMM's last step and this one's first (the conv1 epilogue's h stores).
template <int EXTRA>
__device__ __forceinline__ void chain_gemm(const aw_encoder_chain_args& P, f32x4 (&acc)[4][4], int t0, int T,
                                           const char* smem, uint32_t smem_lds, int tid, const WeightLanes& L,
                                           const f32x4 (&xr)[4][4], rsrc_t xrs, rsrc_t irs) {
  const int w = tid >> 6;
  const uint32_t ring = smem_lds + ACT_BYTES;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < EC_STEPS; ++s) {
    const int t = t0 + s;
    // recompute the lane's addresses every step: hoisted out of the block loop they would pin ~100 VGPRs
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int g = lane >> 4, r = lane & 15;
    if (s < 2)
      step_sync<EXTRA>(t + 1 < T);
    else
      step_sync<0>(t + 1 < T);
    issue_step(P, t + 2, T, ring, L, tid);
    {
      const int i = s >> 2, j = s & 3;
      const int m = 16 * j + (lane & 15), n = 64 * w + 16 * i + (lane >> 4) * 4;
      const int q = s * EC_THREADS + 64 * w + lane, im = q >> 7, ip = q & 127;
      const uint2 iv = *reinterpret_cast<const uint2*>(smem + act_off(im, ip >> 1) + (ip & 1) * 8);
      if (!(EC_PROBE & 1)) {
        store_frag(xrs, (m * EC_H + n) * 4, xr[i][j]);
        store_frag(irs, im * (EC_H * 2) + ip * 8, iv);
      }
    }
    const char* stg = smem + ACT_BYTES + (t % EC_NBUF) * STAGE_BYTES;
    uint4 wf[4], af[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) wf[f] = *reinterpret_cast<const uint4*>(stg + w_off(64 * w + 16 * f + r, g));
#pragma unroll
    for (int f = 0; f < 4; ++f) af[f] = *reinterpret_cast<const uint4*>(smem + act_off(16 * f + r, 4 * s + g));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (!(EC_PROBE & 4))
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[i]),
                                                              __builtin_bit_cast(bf16x8, af[j]), acc[i][j], 0, 0, 0);
  }
  lds_barrier();   // every wave is done with the operand image and the last stage before the epilogue rewrites it
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  const bf16 h[4] = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  uint2 u;
  memcpy(&u, h, 8);
  return u;
}

// bias of channel 64 w + l from the wave's lane l (one VGPR per bias vector, no LDS, no wait in the epilogue)
__device__ __forceinline__ float4 bias4(float bl, int l0) {
  const int v = __float_as_int(bl);
  return make_float4(__int_as_float(__builtin_amdgcn_ds_bpermute(4 * l0, v)),
                     __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (l0 + 1), v)),
                     __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (l0 + 2), v)),
                     __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (l0 + 3), v)));
}

__global__ __launch_bounds__(EC_THREADS, 1) void encoder_chain_kernel(aw_encoder_chain_args P) {
  __shared__ __attribute__((aligned(16))) char smem[EC_LDS];
  const uint32_t smem_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * EC_ROWS;
  const int64_t N = P.N;
  const int R = P.R, T = 32 * R;
  const int rq = (lane >> 4) * 4;     // this lane's 4 channels within a 16-channel fragment
  const int mc = lane & 15;           // this lane's token within a 16-token fragment
  const uint64_t ctr = (P.drop_p > 0.f && P.seed_ptr) ? *P.seed_ptr : 0ull;

  // block-0 operand image (bf16 gelu(x0)), the f32 residual in accumulator layout, the first two ring steps
  {
    const bf16* a0 = reinterpret_cast<const bf16*>(P.a0);
#pragma unroll
    for (int i = 0; i < EC_ROWS * EC_H / 8 / EC_THREADS; ++i) {
      const int q = i * EC_THREADS + tid;
      const int m = q >> 6, c = q & 63;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m0 + m < N) v = *reinterpret_cast<const uint4*>(a0 + (m0 + m) * EC_H + c * 8);
      *reinterpret_cast<uint4*>(smem + act_off(m, c)) = v;
    }
  }
  f32x4 xr[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + 16 * j + mc;
      const int n = 64 * w + 16 * i + rq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < N) v = *reinterpret_cast<const float4*>(P.x0 + m * EC_H + n);
      xr[i][j] = f32x4{v.x, v.y, v.z, v.w};
    }
  const WeightLanes L(tid);
  issue_step(P, 0, T, smem_lds + ACT_BYTES, L, tid);
  issue_step(P, 1, T, smem_lds + ACT_BYTES, L, tid);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // steps 0 and 1 (and every load above) have landed

  f32x4 acc[4][4];
  for (int r = 0; r < R; ++r) {
    const bool last = r == R - 1;
    const float bl1 = P.b1[r][64 * w + lane], bl2 = P.b2[r][64 * w + lane];
    // ---- conv1: h = a . W1^T + b1 -> HBM from the epilogue; a1 = gelu(h) -> the operand image.
    //      Overlapped: x_r and gelu(x_r) of the previous block (outputs x[r-1], aout[r-1]).
    chain_gemm<0>(P, acc, 32 * r, T, smem, smem_lds, tid, L, xr, tile_rsrc(r ? P.x[r - 1] : nullptr, m0, N, EC_H * 4, 8),
                  tile_rsrc(r ? P.aout[r - 1] : nullptr, m0, N, EC_H * 2, 16));
    const rsrc_t hrs = tile_rsrc(P.h[r], m0, N, EC_H * 2, 32);
    {
      // per-lane epilogue addresses recomputed per block (hoisted, they would pin VGPRs across the GEMMs)
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const int rq = (lane >> 4) * 4, mc = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 64 * w + 16 * i + rq;
      const float4 b = bias4(bl1, 16 * i + rq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = 16 * j + mc;
        const float v0 = acc[i][j][0] + b.x, v1 = acc[i][j][1] + b.y, v2 = acc[i][j][2] + b.z,
                    v3 = acc[i][j][3] + b.w;
        if (!(EC_PROBE & 1)) store_frag(hrs, (ml * EC_H + n) * 2, pack4(v0, v1, v2, v3));
        *reinterpret_cast<uint2*>(smem + act_off(ml, n >> 3) + (n & 4) * 2) =
            pack4(gelu_erf_fast(v0), gelu_erf_fast(v1), gelu_erf_fast(v2), gelu_erf_fast(v3));
      }
    }
    }
    // ---- conv2: x += dropout(a1 . W2^T + b2); gelu(x) (x itself after the last block) -> the operand image.
    //      Overlapped: h and a1 of this block.
    chain_gemm<(EC_PROBE & 1) ? 0 : 16>(P, acc, 32 * r + 16, T, smem, smem_lds, tid, L, xr,
                                        tile_rsrc(nullptr, 0, 0, 0), tile_rsrc(P.a1[r], m0, N, EC_H * 2, 16));
    {
      const uint64_t dseed = P.seed_ptr ? aw_seed_mix_value(P.drop_seed[r], ctr) : P.drop_seed[r];
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const int rq = (lane >> 4) * 4, mc = lane & 15;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = 64 * w + 16 * i + rq;
        const float4 b = bias4(bl2, 16 * i + rq);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ml = 16 * j + mc;
          const int64_t m = m0 + ml;
          float v[4] = {acc[i][j][0] + b.x, acc[i][j][1] + b.y, acc[i][j][2] + b.z, acc[i][j][3] + b.w};
          if (P.drop_p > 0.f) {
            float ds[4];
            aw_dropout_scale4(dseed, (uint64_t)m * EC_H + n, P.drop_p, ds);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= ds[e];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) xr[i][j][e] += v[e];
          const f32x4 x = xr[i][j];
          *reinterpret_cast<uint2*>(smem + act_off(ml, n >> 3) + (n & 4) * 2) =
              last ? pack4(x[0], x[1], x[2], x[3])
                   : pack4(gelu_erf_fast(x[0]), gelu_erf_fast(x[1]), gelu_erf_fast(x[2]), gelu_erf_fast(x[3]));
        }
      }
    }
  }
  // tail: x_R and its bf16 image (outputs x[R-1], aout[R-1]) -- nothing left to overlap with
  lds_barrier();
  {
    const rsrc_t xrs = tile_rsrc(P.x[R - 1], m0, N, EC_H * 4), ars = tile_rsrc(P.aout[R - 1], m0, N, EC_H * 2);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int i = s >> 2, j = s & 3;
      const int m = 16 * j + mc, n = 64 * w + 16 * i + rq;
      const int q = s * EC_THREADS + tid, im = q >> 7, ip = q & 127;
      store_frag(xrs, (m * EC_H + n) * 4, xr[i][j]);
      store_frag(ars, im * (EC_H * 2) + ip * 8, *reinterpret_cast<const uint2*>(smem + act_off(im, ip >> 1) +
                                                                                 (ip & 1) * 8));
    }
  }
}

}  // namespace

extern "C" int aw_encoder_chain_fwd(const aw_encoder_chain_args* a, void* stream) {
  AW_REQUIRE(a && a->x0 && a->a0 && a->N >= 0, "aw_encoder_chain_fwd: bad args");
  AW_REQUIRE(a->H == EC_H, "aw_encoder_chain_fwd: H must be %d (got %d)", EC_H, a->H);
  AW_REQUIRE(a->R >= 1 && a->R <= AW_CHAIN_MAX_BLOCKS, "aw_encoder_chain_fwd: 1 <= R <= %d", AW_CHAIN_MAX_BLOCKS);
  AW_REQUIRE(a->drop_p >= 0.f && a->drop_p < 1.f, "aw_encoder_chain_fwd: dropout probability in [0, 1)");
  for (int r = 0; r < a->R; ++r) {
    AW_REQUIRE(a->W1[r] && a->W2[r] && a->b1[r] && a->b2[r], "aw_encoder_chain_fwd: block %d weights missing", r);
    AW_REQUIRE(((uintptr_t)a->W1[r] % 16) == 0 && ((uintptr_t)a->W2[r] % 16) == 0 &&
                   ((uintptr_t)a->b1[r] % 16) == 0 && ((uintptr_t)a->b2[r] % 16) == 0,
               "aw_encoder_chain_fwd: weights and biases must be 16-B aligned");
  }
  AW_REQUIRE(((uintptr_t)a->x0 % 16) == 0 && ((uintptr_t)a->a0 % 16) == 0, "aw_encoder_chain_fwd: unaligned input");
  if (a->N == 0) return AW_OK;
  hipLaunchKernelGGL(encoder_chain_kernel, dim3(aw_cdiv(a->N, EC_ROWS)), dim3(EC_THREADS), 0,
                     reinterpret_cast<hipStream_t>(stream), *a);
  return aw::check_launch("aw_encoder_chain_fwd");
}
