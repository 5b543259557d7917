// MFMA GEMM family for gfx950 (CDNA4): one kernel body for every dense contraction of the hot path.
//
// Tile 128x128 per 256-thread workgroup (4 waves as 2x2, each wave 64x64 = 4x4 fragments of 16x16).
// K is staged through LDS 64 bytes per row per step (32 bf16 or 16 f32), register-staged double buffer,
// one barrier per K step.  Operands are re-laid into a K-contiguous LDS image whatever their global layout,
// so one fragment path serves forward (A.W^T), input-gradient (dY.W) and weight-gradient (dY^T.X) forms and
// the implicit k=3 convolution (row-shifted A or B loads, zero outside each window).
//   bf16: v_mfma_f32_16x16x32_bf16 (fp32 accumulate)      f32: v_mfma_f32_16x16x4_f32 (exact f32)
// Fused epilogue: bias, act' (GELU backward), dropout (counter-based mask), residual add, beta*C,
// second output (act / copy / dropout-masked copy), BatchNorm column statistics, and a fused A-row-sum
// (bias gradients in weight-gradient GEMMs).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, NTHREADS = 256;
constexpr int ROWB = 64;          // bytes of K per LDS row per step
constexpr int PITCHB = ROWB + 16; // padded LDS row pitch in bytes

struct GemmP {
  aw_gemm_args a;
  int tiles_m, tiles_n, nblocks;
};

template <typename T> struct TT;
template <> struct TT<bf16> {
  static constexpr int EPC = 8;                 // elements per 16-byte chunk
  static constexpr int BK = ROWB / 2;           // 32
};
template <> struct TT<float> {
  static constexpr int EPC = 4;
  static constexpr int BK = ROWB / 4;           // 16
};

// One 16-byte chunk of an operand tile, loaded to registers (register staging).
struct Chunk {
  uint4 v;
};

// Load a 16-byte chunk of row-contiguous data at (row, k..k+EPC) -- row-major along K ("k-contiguous").
// Returns zero for out-of-range rows / k and for window-masked implicit-conv rows.
template <typename T>
__device__ __forceinline__ uint4 load_kcontig(const T* base, int64_t ld, int row, int rows_total, int k, int K,
                                              int conv_cin, int conv_seg, int conv_dir) {
  constexpr int EPC = TT<T>::EPC;
  uint4 out = make_uint4(0, 0, 0, 0);
  if (row >= rows_total || k >= K) return out;
  int64_t src_row = row;
  int kk = k;
  if (conv_cin > 0) {
    int j = k / conv_cin;
    kk = k - j * conv_cin;
    int s = conv_dir * (j - 1);
    int t = row % conv_seg;
    if (t + s < 0 || t + s >= conv_seg) return out;
    src_row = row + s;
  }
  const T* p = base + src_row * ld + kk;
  if (k + EPC <= K) {
    out = *reinterpret_cast<const uint4*>(p);
  } else {
    T tmp[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) tmp[e] = (k + e < K) ? p[e] : from_f32<T>(0.f);
    memcpy(&out, tmp, 16);
  }
  return out;
}

// Load a 16-byte chunk of "m-contiguous" data: elements (k, m..m+EPC) of storage [k][m] (ld along k).
// Optional implicit-conv shift along k (rows) with the tap taken from the column index (B operand, wgrad).
template <typename T>
__device__ __forceinline__ uint4 load_mcontig(const T* base, int64_t ld, int k, int K, int m, int Mtot,
                                              int conv_cin, int conv_seg) {
  constexpr int EPC = TT<T>::EPC;
  uint4 out = make_uint4(0, 0, 0, 0);
  if (k >= K || m >= Mtot) return out;
  int64_t src_k = k;
  int mm = m;
  if (conv_cin > 0) {
    int j = m / conv_cin;
    mm = m - j * conv_cin;
    int s = j - 1;
    int t = k % conv_seg;
    if (t + s < 0 || t + s >= conv_seg) return out;
    src_k = k + s;
  }
  const T* p = base + src_k * ld + mm;
  if (m + EPC <= Mtot) {
    out = *reinterpret_cast<const uint4*>(p);
  } else {
    T tmp[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) tmp[e] = (m + e < Mtot) ? p[e] : from_f32<T>(0.f);
    memcpy(&out, tmp, 16);
  }
  return out;
}

// Stage one operand tile (128 rows x BK) into registers: 2 chunks per thread.
template <typename T>
__device__ __forceinline__ void stage_load(Chunk (&c)[2], const T* base, int64_t ld, int trans, int row0,
                                           int rows_total, int k0, int K, int conv_cin, int conv_seg,
                                           int conv_dir, int tid) {
  constexpr int EPC = TT<T>::EPC;
  constexpr int BK = TT<T>::BK;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int ci = tid + i * NTHREADS;
    if (!trans) {  // k-contiguous: 4 chunks per row
      int r = ci >> 2, kc = ci & 3;
      c[i].v = load_kcontig<T>(base, ld, row0 + r, rows_total, k0 + kc * EPC, K, conv_cin, conv_seg, conv_dir);
    } else {       // row-contiguous: 128/EPC chunks per k-row
      constexpr int CPR = 128 / EPC;
      int kr = ci / CPR, mc = ci % CPR;
      c[i].v = load_mcontig<T>(base, ld, k0 + kr, K, row0 + mc * EPC, rows_total, conv_cin, conv_seg);
    }
  }
  (void)BK;
}

template <typename T>
__device__ __forceinline__ void stage_store(const Chunk (&c)[2], char* lds, int trans, int tid) {
  constexpr int EPC = TT<T>::EPC;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int ci = tid + i * NTHREADS;
    if (!trans) {
      int r = ci >> 2, kc = ci & 3;
      *reinterpret_cast<uint4*>(lds + r * PITCHB + kc * 16) = c[i].v;
    } else {
      constexpr int CPR = 128 / EPC;
      int kr = ci / CPR, mc = ci % CPR;
      T tmp[EPC];
      memcpy(tmp, &c[i].v, 16);
#pragma unroll
      for (int e = 0; e < EPC; ++e)
        *reinterpret_cast<T*>(lds + (mc * EPC + e) * PITCHB + kr * (int)sizeof(T)) = tmp[e];
    }
  }
}

template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
  __device__ __forceinline__ static void run(f32x4& acc, const uint4& a, const uint4& b) {
    bf16x8 av, bv;
    memcpy(&av, &a, 16);
    memcpy(&bv, &b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  __device__ __forceinline__ static void run(f32x4& acc, const uint4& a, const uint4& b) {
    f32x4 av, bv;
    memcpy(&av, &a, 16);
    memcpy(&bv, &b, 16);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
  }
};

__device__ __forceinline__ float act_fwd(int act, float x) { return act == AW_ACT_GELU_TANH ? gelu_tanh(x) : gelu_erf(x); }
__device__ __forceinline__ float act_bwd(int act, float x) {
  return act == AW_ACT_GELU_TANH ? gelu_tanh_grad(x) : gelu_erf_grad(x);
}

// Bijective XCD-aware remap: consecutive logical tiles land on the same XCD (blocks b and b+8 share one).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  int q = nblocks / 8, r = nblocks % 8;
  int xcd = bid % 8, slot = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

template <typename T>
__global__ __launch_bounds__(NTHREADS) void gemm_kernel(GemmP P) {
  constexpr int BK = TT<T>::BK;
  constexpr int EPC = TT<T>::EPC;
  const aw_gemm_args& p = P.a;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 128 * PITCHB];
  // stage buffer b: A image at smem + b*STAGE, B image right after it
  constexpr int STAGE = 2 * 128 * PITCHB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tile = xcd_remap(blockIdx.x, P.nblocks);
  const int tm = tile / P.tiles_n, tn = tile % P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int M = p.M, N = p.N, K = p.K;

  const T* Ab = reinterpret_cast<const T*>(p.A);
  const T* Bb = reinterpret_cast<const T*>(p.B);
  const int a_conv = (p.conv_cin > 0 && p.conv_operand == 0) ? p.conv_cin : 0;
  const int b_conv = (p.conv_cin > 0 && p.conv_operand == 1) ? p.conv_cin : 0;
  const bool do_rowsum = p.a_rowsum != nullptr && tn == 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rowsum = 0.f;

  const int nk = (K + BK - 1) / BK;
  Chunk ca[2], cb[2];
  stage_load<T>(ca, Ab, p.lda, p.a_trans, m0, M, 0, K, a_conv, p.conv_seg, p.conv_dir, tid);
  stage_load<T>(cb, Bb, p.ldb, p.b_trans, n0, N, 0, K, b_conv, p.conv_seg, 1, tid);
  stage_store<T>(ca, smem, p.a_trans, tid);
  stage_store<T>(cb, smem + 128 * PITCHB, p.b_trans, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      stage_load<T>(ca, Ab, p.lda, p.a_trans, m0, M, (kt + 1) * BK, K, a_conv, p.conv_seg, p.conv_dir, tid);
      stage_load<T>(cb, Bb, p.ldb, p.b_trans, n0, N, (kt + 1) * BK, K, b_conv, p.conv_seg, 1, tid);
    }
    const char* a_l = smem + cur * STAGE;
    const char* b_l = a_l + 128 * PITCHB;
    uint4 af[4], bfr[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      af[f] = *reinterpret_cast<const uint4*>(a_l + (wm * 64 + f * 16 + (lane & 15)) * PITCHB + (lane >> 4) * 16);
      bfr[f] = *reinterpret_cast<const uint4*>(b_l + (wn * 64 + f * 16 + (lane & 15)) * PITCHB + (lane >> 4) * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) Mfma<T>::run(acc[i][j], af[i], bfr[j]);
    if (do_rowsum) {  // row r = tid>>1 sums half a K step
      const T* rowp = reinterpret_cast<const T*>(a_l + (tid >> 1) * PITCHB) + (tid & 1) * (BK / 2);
#pragma unroll
      for (int e = 0; e < BK / 2; ++e) rowsum += to_f32<T>(rowp[e]);
    }
    if (kt + 1 < nk) {
      stage_store<T>(ca, smem + (cur ^ 1) * STAGE, p.a_trans, tid);
      stage_store<T>(cb, smem + (cur ^ 1) * STAGE + 128 * PITCHB, p.b_trans, tid);
    }
    __syncthreads();
  }
  (void)EPC;

  if (do_rowsum) {
    rowsum += __shfl_xor(rowsum, 1, 64);
    int r = m0 + (tid >> 1);
    if ((tid & 1) == 0 && r < M) atomicAdd(p.a_rowsum + r, rowsum);
  }

  // ---------------------------------------------------------------- epilogue
  const int cq = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + j * 16 + cq;
    const bool col_ok = col < N;
    const float bias = (p.bias && col_ok) ? p.bias[p.bias_mod > 0 ? col % p.bias_mod : col] : 0.f;
    float csum = 0.f, csq = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + rq + r;
        if (!col_ok || row >= M) continue;
        float v = p.alpha * acc[i][j][r] + bias;
        if (p.pre) v *= act_bwd(p.act, p.pre[(int64_t)row * p.ld_pre + col]);
        if (p.drop_p > 0.f) v *= aw_dropout_scale(p.drop_seed, (uint64_t)row * N + col, p.drop_p);
        if (p.resid) v += p.resid[(int64_t)row * p.ld_resid + col];
        if (p.beta != 0.f) v += p.beta * reinterpret_cast<const float*>(p.C)[(int64_t)row * p.ldc + col];
        if (p.C) store_from_f32(p.C, p.c_dtype, (int64_t)row * p.ldc + col, v);
        if (p.c2_mode) {
          float w = v;
          if (p.c2_mode == 1) w = act_fwd(p.act, v);
          else if (p.c2_mode == 3) w = v * aw_dropout_scale(p.drop2_seed, (uint64_t)row * N + col, p.drop2_p);
          store_from_f32(p.C2, p.c2_dtype, (int64_t)row * p.ldc2 + col, w);
        }
        csum += v;
        csq += v * v;
      }
    }
    if (p.colstats) {
      // reduce over the 4 row-quads of the wave (lanes with equal lane&15)
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      csq += __shfl_xor(csq, 16, 64);
      csq += __shfl_xor(csq, 32, 64);
      if (lane < 16 && col_ok) {
        int s = col % p.stats_mod;
        atomicAdd(p.colstats + s, (double)csum);
        atomicAdd(p.colstats + p.stats_mod + s, (double)csq);
      }
    }
  }
}

}  // namespace

extern "C" int aw_gemm(const aw_gemm_args* args, void* stream) {
  if (!args) {
    aw::set_error("aw_gemm: null args");
    return AW_ERR_ARG;
  }
  const aw_gemm_args& a = *args;
  AW_REQUIRE(a.M >= 0 && a.N >= 0 && a.K >= 0, "aw_gemm: negative size");
  AW_REQUIRE(a.a_dtype == AW_F32 || a.a_dtype == AW_BF16, "aw_gemm: bad a_dtype %d", a.a_dtype);
  AW_REQUIRE(a.A && a.B, "aw_gemm: null operand");
  const int epc = a.a_dtype == AW_BF16 ? 8 : 4;
  AW_REQUIRE(((uintptr_t)a.A % 16) == 0 && ((uintptr_t)a.B % 16) == 0, "aw_gemm: operands must be 16-B aligned");
  AW_REQUIRE(a.lda % epc == 0 && a.ldb % epc == 0, "aw_gemm: lda/ldb must be multiples of %d elements", epc);
  if (a.conv_cin > 0) {
    AW_REQUIRE(a.conv_seg > 0 && a.conv_cin % epc == 0, "aw_gemm: conv_cin must be a multiple of %d", epc);
    if (a.conv_operand == 0)
      AW_REQUIRE(a.a_trans == 0 && a.K == 3 * a.conv_cin, "aw_gemm: A-conv needs a_trans=0 and K=3*cin");
    else
      AW_REQUIRE(a.b_trans == 1 && a.N == 3 * a.conv_cin, "aw_gemm: B-conv needs b_trans=1 and N=3*cin");
  }
  AW_REQUIRE(!(a.beta != 0.f && a.c_dtype != AW_F32), "aw_gemm: beta != 0 needs an f32 C");
  AW_REQUIRE(!(a.c2_mode && !a.C2), "aw_gemm: c2_mode without C2");
  AW_REQUIRE(!(a.colstats && a.stats_mod <= 0), "aw_gemm: colstats needs stats_mod > 0");
  if (a.M == 0 || a.N == 0) return AW_OK;
  GemmP P;
  P.a = a;
  P.tiles_m = aw_cdiv(a.M, BM);
  P.tiles_n = aw_cdiv(a.N, BN);
  P.nblocks = P.tiles_m * P.tiles_n;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.a_dtype == AW_BF16)
    hipLaunchKernelGGL(gemm_kernel<bf16>, dim3(P.nblocks), dim3(NTHREADS), 0, s, P);
  else
    hipLaunchKernelGGL(gemm_kernel<float>, dim3(P.nblocks), dim3(NTHREADS), 0, s, P);
  return aw::check_launch("aw_gemm");
}
