// MFMA GEMM family: host entry points (aw_gemm, aw_gemm_ws, aw_gemm_workspace) and the EP_GENERIC / EP_ACCUM
// kernel instantiations.  The kernel itself is in gemm_core.h; specialised epilogues in gemm_fast_*.hip.
#include <stdlib.h>

#include "gemm_core.h"

using namespace awg;

namespace {

template <typename T, Layout LY>
void launch_generic(const GemmP& P, hipStream_t s, bool ragged) {
  if (ragged) launch_kernel<T, LY, true, EP_GENERIC, 128>(P, s);
  else launch_tiled<T, LY, EP_GENERIC>(P, s);
}

Layout layout_of(const aw_gemm_args& a) {
  const bool conv = a.conv_cin > 0;
  const bool aconv = conv && a.conv_operand == 0, bconv = conv && a.conv_operand == 1;
  if (!a.a_trans && !a.b_trans) return aconv ? L_NN_CONV : L_NN;
  if (!a.a_trans && a.b_trans) return aconv ? L_NT_CONV : L_NT;
  if (a.a_trans && !a.b_trans) return L_TN;
  return bconv ? L_TT_KCONV : L_TT;
}

// compile-time epilogue code of a launch (EP_GENERIC when no specialisation can apply)
uint32_t epi_code(const aw_gemm_args& a, const GemmP& P, bool ragged) {
  if (P.splits > 1 || a.accumulate) return ragged ? EP_GENERIC : EP_ACCUM;
  if (ragged || !P.vec || a.N % 4 != 0 || a.alpha != 1.f) return EP_GENERIC;
  uint32_t c = 0;
  if (a.bias) c |= EP_BIAS;
  if (a.bias && a.bias_mod > 0) c |= EP_BIASMOD;
  if (a.pre) c |= EP_PRE | (a.pre_dtype == AW_BF16 ? EP_PREBF : 0u);
  if ((a.pre || a.c2_mode == 1 || a.c2_mode == 4) && a.act == AW_ACT_GELU_TANH) c |= EP_TANH;
  if (a.pre && a.act == AW_ACT_DERIV) c |= EP_DERIV;
  if (a.drop_p > 0.f) c |= EP_DROP;
  if (a.resid) c |= EP_RESID | (a.resid_dtype == AW_BF16 ? EP_RESIDBF : 0u);
  if (a.beta != 0.f) c |= EP_BETA;
  if (a.C) c |= EP_C | (a.c_dtype == AW_BF16 ? EP_CBF : 0u);
  if (a.c2_mode == 1) c |= EP_C2ACT;
  else if (a.c2_mode == 2 || (a.c2_mode == 3 && a.drop2_p <= 0.f)) c |= EP_C2COPY;
  else if (a.c2_mode == 3) c |= EP_C2DROP;
  else if (a.c2_mode == 4) c |= EP_C2DACT;
  if (a.c2_mode && a.c2_dtype == AW_BF16) c |= EP_C2BF;
  if (a.colstats) c |= EP_STATS;
  return c;
}

template <typename T>
void dispatch(const GemmP& P, hipStream_t s, bool ragged) {
  const Layout ly = layout_of(P.a);
  uint32_t code = epi_code(P.a, P, ragged);
  constexpr bool BF = sizeof(T) == 2;
  if (code == EP_ACCUM) {
    switch (ly) {
      case L_TN: launch_tiled<T, L_TN, EP_ACCUM>(P, s); return;
      case L_TT: launch_tiled<T, L_TT, EP_ACCUM>(P, s); return;
      case L_TT_KCONV: launch_tiled<T, L_TT_KCONV, EP_ACCUM>(P, s); return;
      default: break;
    }
  } else if (code != EP_GENERIC) {
    if ((ly == L_NN || ly == L_NN_CONV) && launch_fast_fwd(P, s, BF, ly, code)) return;
    if ((ly == L_NT || ly == L_NT_CONV) && launch_fast_bwd(P, s, BF, ly, code)) return;
  }
  switch (ly) {
    case L_NN: launch_generic<T, L_NN>(P, s, ragged); break;
    case L_NN_CONV: launch_generic<T, L_NN_CONV>(P, s, ragged); break;
    case L_NT: launch_generic<T, L_NT>(P, s, ragged); break;
    case L_NT_CONV: launch_generic<T, L_NT_CONV>(P, s, ragged); break;
    case L_TN: launch_generic<T, L_TN>(P, s, ragged); break;
    case L_TT: launch_generic<T, L_TT>(P, s, ragged); break;
    case L_TT_KCONV: launch_generic<T, L_TT_KCONV>(P, s, ragged); break;
  }
}


// sum of the split-K slabs -> C (accumulate mode: += through the column map; else alpha*sum + beta*C).
// Four consecutive elements per thread (N % 4 == 0: float4 slab loads) and four independent partial sums over the
// splits, so a thread keeps its slab loads in flight instead of waiting on one add chain per split.
__device__ __forceinline__ void reduce_store(const aw_gemm_args& p, float* C, int64_t r, int c, float acc) {
  if (p.accumulate) {
    const int64_t oc = p.col_mod > 0 ? (int64_t)(c % p.col_mod) * p.col_mul + c / p.col_mod + p.col_off
                                     : (int64_t)c * (p.col_mul > 0 ? p.col_mul : 1) + p.col_off;
    C[r * p.ldc + oc] += p.alpha * acc;
  } else {
    float v = p.alpha * acc;
    if (p.beta != 0.f) v += p.beta * C[r * p.ldc + c];
    C[r * p.ldc + c] = v;
  }
}

__global__ __launch_bounds__(256) void gemm_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                          aw_gemm_args p) {
  const int64_t n = (int64_t)M * N;
  float* C = reinterpret_cast<float*>(p.C);
  if (p.accumulate && p.col_mod > 0 && (int64_t)p.col_mod * p.col_mul == N && (N & 3) == 0 && (p.ldc & 3) == 0 &&
      (p.col_off & 3) == 0 && ((uintptr_t)C & 15) == 0) {
    // transposing column map (ConvT weight gradient: column j*col_mod + o lands at o*col_mul + j): walk the
    // DESTINATION in float4s so the read-modify-write of C is coalesced; the slab reads gather col_mul runs of
    // consecutive o per wave instead
    const int64_t n4 = n >> 2;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
      const int64_t e = q << 2;
      const int64_t r = e / N;
      const int d0 = (int)(e - r * N);
      int64_t src[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = d0 + k, o = d / p.col_mul, j = d - o * p.col_mul;
        src[k] = r * N + (int64_t)j * p.col_mod + o;
      }
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < splits; ++s) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += ws[s * n + src[k]];
      }
      f32x4* dst = reinterpret_cast<f32x4*>(C + r * p.ldc + p.col_off + d0);
      f32x4 v = *dst;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += p.alpha * acc[k];
      *dst = v;
    }
    return;
  }
  if ((N & 3) == 0) {
    const int64_t n4 = n >> 2;
    const f32x4* w4 = reinterpret_cast<const f32x4*>(ws);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
      int s = 0;
      for (; s + 4 <= splits; s += 4) {
        a0 += w4[(s + 0) * n4 + q];
        a1 += w4[(s + 1) * n4 + q];
        a2 += w4[(s + 2) * n4 + q];
        a3 += w4[(s + 3) * n4 + q];
      }
      for (; s < splits; ++s) a0 += w4[s * n4 + q];
      const f32x4 acc = (a0 + a1) + (a2 + a3);
      const int64_t e = q << 2;
      const int64_t r = e / N;
      const int c = (int)(e - r * N);
#pragma unroll
      for (int k = 0; k < 4; ++k) reduce_store(p, C, r, c + k, acc[k]);
    }
    return;
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += ws[s * n + e];
    const int64_t r = e / N;
    reduce_store(p, C, r, (int)(e - r * N), acc);
  }
}

}  // namespace

extern "C" int aw_gemm_ws(const aw_gemm_args* args, float* ws, int64_t ws_elems, void* stream);

extern "C" int aw_gemm(const aw_gemm_args* args, void* stream) { return aw_gemm_ws(args, nullptr, 0, stream); }

// argument checks shared by aw_gemm_ws and aw_gemm_grouped
static int validate(const aw_gemm_args& a) {
  AW_REQUIRE(a.M >= 0 && a.N >= 0 && a.K >= 0, "aw_gemm: negative size");
  AW_REQUIRE(a.a_dtype == AW_F32 || a.a_dtype == AW_BF16, "aw_gemm: bad a_dtype %d", a.a_dtype);
  AW_REQUIRE(a.A && a.B, "aw_gemm: null operand");
  const int epc = a.a_dtype == AW_BF16 ? 8 : 4;
  const int BK = a.a_dtype == AW_BF16 ? 64 : 32;
  AW_REQUIRE(((uintptr_t)a.A % 16) == 0 && ((uintptr_t)a.B % 16) == 0, "aw_gemm: operands must be 16-B aligned");
  AW_REQUIRE(a.lda % epc == 0 && a.ldb % epc == 0, "aw_gemm: lda/ldb must be multiples of %d elements", epc);
  if (a.conv_cin > 0) {
    AW_REQUIRE(a.conv_seg > 0 && a.conv_cin % epc == 0, "aw_gemm: conv_cin must be a multiple of %d", epc);
    if (a.conv_operand == 0)
      AW_REQUIRE(a.a_trans == 0 && a.K == 3 * a.conv_cin, "aw_gemm: A-conv needs a_trans=0 and K=3*cin");
    else
      AW_REQUIRE(a.a_trans == 1 && a.b_trans == 1 && a.N == 3 * a.conv_cin,
                 "aw_gemm: B-conv needs a_trans=1, b_trans=1 and N=3*cin");
    AW_REQUIRE(a.conv_cin % BK == 0, "aw_gemm: conv_cin must be a multiple of %d", BK);
  }
  AW_REQUIRE(!(a.beta != 0.f && a.c_dtype != AW_F32), "aw_gemm: beta != 0 needs an f32 C");
  AW_REQUIRE(!(a.c2_mode && !a.C2), "aw_gemm: c2_mode without C2");
  AW_REQUIRE(a.c2_mode >= 0 && a.c2_mode <= 4 && a.act >= AW_ACT_GELU_ERF && a.act <= AW_ACT_DERIV,
             "aw_gemm: bad c2_mode %d / act %d", a.c2_mode, a.act);
  AW_REQUIRE(!(a.act == AW_ACT_DERIV && (a.c2_mode == 1 || a.c2_mode == 4)),
             "aw_gemm: AW_ACT_DERIV names no activation for C2 modes 1 / 4");
  AW_REQUIRE(!(a.colstats && a.stats_mod <= 0), "aw_gemm: colstats needs stats_mod > 0");
  AW_REQUIRE(a.pre_dtype == AW_F32 || a.pre_dtype == AW_BF16, "aw_gemm: bad pre_dtype %d", a.pre_dtype);
  AW_REQUIRE(a.resid_dtype == AW_F32 || a.resid_dtype == AW_BF16, "aw_gemm: bad resid_dtype %d", a.resid_dtype);
  AW_REQUIRE(a.store_policy == AW_STORE_NT || a.store_policy == AW_STORE_WT, "aw_gemm: bad store_policy %d",
             a.store_policy);
  const bool plain = !a.bias && !a.pre && !a.resid && a.drop_p <= 0.f && !a.C2 && !a.colstats && a.C &&
                     a.c_dtype == AW_F32 && (a.beta == 0.f || a.beta == 1.f || a.accumulate);
  AW_REQUIRE(!a.accumulate || plain, "aw_gemm: accumulate mode allows no other epilogue field (f32 C only)");
  AW_REQUIRE(!(a.accumulate && a.beta != 0.f), "aw_gemm: accumulate mode already adds into C (beta must be 0)");
  {
    const int64_t es = a.a_dtype == AW_BF16 ? 2 : 4;
    const int64_t ka = a.K > 0 ? a.K : 1;
    const int64_t ea = (!a.a_trans ? ((int64_t)(a.M - 1) * a.lda + ka) : ((ka - 1) * a.lda + a.M)) * es;
    const int64_t eb = (!a.b_trans ? ((int64_t)(a.N - 1) * a.ldb + ka) : ((ka - 1) * a.ldb + a.N)) * es;
    AW_REQUIRE(ea < OOB && eb < OOB, "aw_gemm: operand extent >= 2 GiB is not supported");
  }
  return AW_OK;
}

// ragged: a contiguous extent that is not a whole number of 16-B chunks.  A row-contiguous (transposed) operand
// whose leading dimension is padded to whole chunks is not ragged: the over-read lanes only feed output rows /
// columns >= M / N, which are never stored (e.g. the patch-embed weight gradient, N = P = 25, ldb = 32).
static bool is_ragged(const aw_gemm_args& a) {
  const int epc = a.a_dtype == AW_BF16 ? 8 : 4;
  auto padded = [epc](int n, int64_t ld) { return ld >= (int64_t)(n + epc - 1) / epc * epc; };
  const bool ra = !a.a_trans ? (a.K % epc) != 0 : (a.M % epc != 0 && !padded(a.M, a.lda));
  const bool rb = !a.b_trans ? (a.K % epc) != 0 : (a.N % epc != 0 && !padded(a.N, a.ldb));
  return ra || rb;
}

// most split-K slices of one grouped weight-gradient tile (their partials meet in the epilogue's f32 atomics)
// (8: the transformer's four 512 x 512 projections, 64 tiles, take 63 instead of 103 us; the wider kinds already fill
// the chip with two slices)
#ifndef AW_GROUPED_MAXSPLIT
#define AW_GROUPED_MAXSPLIT 8
#endif

// fewest K steps of one split-K slice of a plain 128-tile launch (its slab write + reduce stay small against them)
#ifndef AW_SPLIT_MIN_KSTEPS
#define AW_SPLIT_MIN_KSTEPS 12
#endif

// fewest K steps of one split of a launch with at most 16 output tiles (the VQ-VAE's small weight gradients: M x N =
// 512 x 25 / 64 x 512 / 512 x 64 over K = 16384 tokens): 6 (tools/probe/small_wgrad_probe.py, same box: 24.1 / 18.7 /
// 19.7 us at 12, 24.2 / 17.0 / 17.8 at 6, 29.1 / 18.0 / 19.2 at 4); AW_SPLIT_MIN_KSTEPS_SMALL: tuning override
static int min_ksteps_small() {
  static const int v = [] {
    const char* e = getenv("AW_SPLIT_MIN_KSTEPS_SMALL");
    return e && atoi(e) > 0 ? atoi(e) : 6;
  }();
  return v;
}

static int g_tile_override = 0;   // aw_gemm_set_tile: 0 = automatic, 128 / 256 = force (tests, tuning)

extern "C" int aw_gemm_set_tile(int bm) {
  AW_REQUIRE(bm == 0 || bm == 128 || bm == 256, "aw_gemm_set_tile: bm must be 0, 128 or 256");
  g_tile_override = bm;
  return AW_OK;
}

static bool plain_output(const aw_gemm_args& a) {
  return !a.bias && !a.pre && !a.resid && a.drop_p <= 0.f && !a.C2 && !a.colstats && a.C && a.c_dtype == AW_F32 &&
         (a.beta == 0.f || a.beta == 1.f || a.accumulate);
}

// Launch plan of ngroups problems of one shape: tile (128 or 256 rows), grid and split-K.
//  * 128x128 tiles, two workgroups per CU (measured equal or faster than the 256x128 three-stage tile on every
//    shape of the path: forward / input-gradient M = 16384, K = 512 .. 2048 and the grouped weight gradients);
//    plain f32 outputs that cannot fill the chip twice are split over K (slab workspace when the caller provides
//    one, f32 atomics in grouped launches, <= 2 adders);
//  * 256x128 ping-pong tiles, one workgroup per CU, for bf16 launches whose 256-row tiles fill the chip
//    (aw_gemm_set_tile(256) forces them for every eligible bf16 launch, (128) disables them).
static void plan(const aw_gemm_args& a, int ngroups, bool grouped, GemmP& P) {
  P.a = a;
  P.ngroups = ngroups;
  P.ws = nullptr;
  auto al = [](const void* ptr, int64_t ld, int dt) {
    return ptr == nullptr || (((uintptr_t)ptr % 16) == 0 && (ld * (dt == AW_BF16 ? 2 : 4)) % 16 == 0);
  };
  P.vec = al(a.C, a.ldc, a.c_dtype) && al(a.C2, a.ldc2, a.c2_dtype) && al(a.pre, a.ld_pre, a.pre_dtype) &&
          al(a.resid, a.ld_resid, a.resid_dtype);
  const int64_t es = a.a_dtype == AW_BF16 ? 2 : 4;
  const int64_t ka = a.K > 0 ? a.K : 1;
  // a padded transposed operand is read in whole chunks up to its padded width (see is_ragged)
  const int epc = a.a_dtype == AW_BF16 ? 8 : 4;
  auto wide = [epc](int n, int64_t ld) { const int64_t r = (int64_t)(n + epc - 1) / epc * epc; return ld >= r ? r : n; };
  P.a_bytes = (int)((!a.a_trans ? ((int64_t)(a.M - 1) * a.lda + ka) : ((ka - 1) * a.lda + wide(a.M, a.lda))) * es);
  P.b_bytes = (int)((!a.b_trans ? ((int64_t)(a.N - 1) * a.ldb + ka) : ((ka - 1) * a.ldb + wide(a.N, a.ldb))) * es);

  const int BK = a.a_dtype == AW_BF16 ? 64 : 32;
  const bool plain = plain_output(a);
  P.tiles_n = aw_cdiv(a.N, BN);
  const int t256 = aw_cdiv(a.M, 256) * P.tiles_n * ngroups;
  int bm = 128, splits = 1;
  // 256-row ping-pong tiles (one workgroup per CU) for the bf16 forward layouts (both operands K-contiguous) whose
  // 256-row tiles alone fill the chip and that run at least 16 K steps: the decoder convs (K = 1536; same-box A/B
  // 35.6 / 44.9 vs 38.4 / 46.0 us).  The input-gradient layouts (transposed weight reads) and the K = 512 encoder
  // convs measured slower on the 256-row tile (e.g. 54.1 vs 51.0 us, 33.3 vs 31.5 us) and keep the 128-row form.
  // aw_gemm_set_tile(128) keeps every launch on the 128-row form, (256) forces the 256-row tile where eligible.
  const bool auto256 = t256 >= 256 && !grouped && !a.accumulate && !a.a_trans && !a.b_trans && a.K >= 16 * BK;
  if (a.a_dtype == AW_BF16 && !is_ragged(a) && (g_tile_override == 256 || (g_tile_override == 0 && auto256))) {
    bm = 256;
    if (a.accumulate && t256 < 240 && a.K >= 24 * BK) {
      splits = 256 / t256;
      if (splits > a.K / (12 * BK)) splits = a.K / (12 * BK);
      if (grouped && splits > AW_GROUPED_MAXSPLIT) splits = AW_GROUPED_MAXSPLIT;
      if (splits < 1) splits = 1;
    }
  }
  if (bm == 128) {
    const int nb = aw_cdiv(a.M, 128) * P.tiles_n * ngroups;
    if (plain && nb < 384 && a.K >= 24 * BK) {
      // two co-resident blocks per CU (256 CUs); keep >= 12 K-steps per split so the slab write + reduce is small
      splits = 512 / nb;
      const int max_splits = a.K / ((nb <= 16 ? min_ksteps_small() : AW_SPLIT_MIN_KSTEPS) * BK);
      if (splits > max_splits) splits = max_splits;
      if (grouped && splits > AW_GROUPED_MAXSPLIT) splits = AW_GROUPED_MAXSPLIT;
      if (splits < 1) splits = 1;
    }
    if (grouped && a.accumulate && nb > 512 && nb < 1024 && a.K >= 48 * BK) {
      // 1.5 waves of 128-tiles (the decoder weight gradients: 768) -> 3 full waves of half-K units; the halves
      // meet in the accumulating atomics the epilogue issues anyway (same-box A/B: +1.3 % windows/s)
      splits = 2;
    }
  }
  P.bm = bm;
  P.tiles_per_group = aw_cdiv(a.M, bm) * P.tiles_n;
  P.nblocks = P.tiles_per_group * ngroups;
  P.ksplit = splits > 1 ? aw_cdiv(aw_cdiv(a.K, splits), BK) * BK : (a.K > 0 ? a.K : 1);
  P.splits = splits > 1 ? aw_cdiv(a.K, P.ksplit) : 1;
}

// the slab workspace is used by single 128-tile launches split over K (grouped and 256-tile splits use atomics)
static bool wants_slabs(const aw_gemm_args& a, const GemmP& P) { return P.splits > 1 && P.bm == 128 && (a.beta == 0.f || a.beta == 1.f || a.accumulate); }

extern "C" int64_t aw_gemm_workspace(const aw_gemm_args* a) {
  if (!a || a->M <= 0 || a->N <= 0) return 0;
  GemmP P;
  plan(*a, 1, false, P);
  return wants_slabs(*a, P) ? (int64_t)P.splits * a->M * a->N : 0;
}

extern "C" int aw_gemm_ws(const aw_gemm_args* args, float* ws, int64_t ws_elems, void* stream) {
  if (!args) {
    aw::set_error("aw_gemm: null args");
    return AW_ERR_ARG;
  }
  const aw_gemm_args& a = *args;
  if (int st = validate(a)) return st;
  if (a.M == 0 || a.N == 0) return AW_OK;
  GemmP P;
  plan(a, 1, false, P);
  if (wants_slabs(a, P) && ws && ws_elems >= (int64_t)P.splits * a.M * a.N) P.ws = ws;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (P.splits > 1 && !P.ws && a.beta == 0.f && !a.accumulate) {   // atomics into a zeroed C
    if (hipMemset2DAsync(a.C, a.ldc * sizeof(float), 0, a.N * sizeof(float), a.M, s) != hipSuccess)
      return aw::check_launch("aw_gemm split-K zero");
  }
  const bool ragged = is_ragged(a);
  if (a.a_dtype == AW_BF16)
    dispatch<bf16>(P, s, ragged);
  else
    dispatch<float>(P, s, ragged);
  if (P.ws) {
    const int64_t n = (int64_t)a.M * a.N;
    int64_t g = ((a.N & 3) == 0 ? n / 4 + 255 : n + 255) / 256;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(gemm_reduce_kernel, dim3((int)g), dim3(256), 0, s, P.ws, P.splits, a.M, a.N, a);
  }
  return aw::check_launch("aw_gemm");
}

extern "C" int aw_gemm_grouped(const aw_gemm_args* args, int n, void* stream) {
  AW_REQUIRE(args && n >= 1 && n <= AW_GEMM_MAX_GROUPS, "aw_gemm_grouped: need 1..%d problems", AW_GEMM_MAX_GROUPS);
  const aw_gemm_args& a = args[0];
  for (int g = 0; g < n; ++g) {
    if (int st = validate(args[g])) return st;
    const aw_gemm_args& b = args[g];
    // every field but the four per-group pointers must match problem 0
    const bool same = b.M == a.M && b.N == a.N && b.K == a.K && b.a_dtype == a.a_dtype && b.lda == a.lda &&
                      b.a_trans == a.a_trans && b.ldb == a.ldb && b.b_trans == a.b_trans &&
                      b.conv_cin == a.conv_cin && b.conv_seg == a.conv_seg && b.conv_dir == a.conv_dir &&
                      b.conv_operand == a.conv_operand && b.alpha == a.alpha && b.beta == a.beta &&
                      b.ldc == a.ldc && b.c_dtype == a.c_dtype && b.accumulate == a.accumulate &&
                      b.col_mod == a.col_mod && b.col_mul == a.col_mul && b.col_off == a.col_off &&
                      (b.a_rowsum == nullptr) == (a.a_rowsum == nullptr) && b.C != nullptr;
    AW_REQUIRE(same, "aw_gemm_grouped: problem %d differs from problem 0 in more than A, B, C, a_rowsum", g);
  }
  AW_REQUIRE(a.accumulate && !a.C2 && !a.bias && !a.colstats, "aw_gemm_grouped: accumulate-mode problems only");
  if (a.M == 0 || a.N == 0) return AW_OK;
  if (wgrad_conv3_try(args, n, reinterpret_cast<hipStream_t>(stream))) return aw::check_launch("aw_gemm_grouped");
  GemmP P;
  plan(a, n, true, P);
  for (int g = 0; g < n; ++g) {
    P.gA[g] = args[g].A;
    P.gB[g] = args[g].B;
    P.gC[g] = args[g].C;
    P.gRow[g] = args[g].a_rowsum;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool ragged = is_ragged(a);
  if (a.a_dtype == AW_BF16)
    dispatch<bf16>(P, s, ragged);
  else
    dispatch<float>(P, s, ragged);
  return aw::check_launch("aw_gemm_grouped");
}
