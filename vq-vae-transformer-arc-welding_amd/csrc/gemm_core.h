// MFMA GEMM family for gfx950 (CDNA4): one kernel body for every dense contraction of the hot path.
//
// Two tile configurations (template BMT):
//   BMT = 128: 128x128 tile, 256 threads (4 waves as 2x2), two LDS stages, two workgroups per CU;
//   BMT = 256: 256x128 tile, 512 threads (8 waves as 4x2), three LDS stages, one workgroup per CU, the two wave
//              groups ping-ponging between fragment reads + DMA issue and MFMAs (see the main loop).
// Every wave owns a 64x64 output block = 4x4 fragments of 16x16.  K is staged 128 bytes per operand row per step
// (64 bf16 / 32 f32).  Operands reach LDS by LDS-DMA (gfx950 `buffer_load ... lds`): the image swizzle is applied
// to the source address, out-of-range offsets implement every mask (M/N/K tails, implicit-conv window edges).
// Ragged shapes (a contiguous extent that is not whole 16-B chunks) use register staging instead.
// Operand layouts are compile-time template parameters:
//   K-contiguous operand ([rows][K], e.g. activations in forward, weights [out][in]) -> LDS image [row][k],
//       16-B chunks XOR-swizzled per row pair, fragments by one ds_read_b128;
//   row-contiguous operand ([K][rows], e.g. activations as the weight-gradient reduction operand) -> LDS image
//       [k][row] with a per-k-row rotation; bf16 fragments come from two ds_read_b64_tr_b16 hardware-transposed
//       reads (gfx950), f32 fragments from four ds_read_b32.
// Implicit k=3/pad=1 convolution (decoder ResBlocks) = row-shifted loads with a per-window zero mask.
//   bf16: v_mfma_f32_16x16x32_bf16 (fp32 accumulate)      f32: v_mfma_f32_16x16x4_f32 (exact f32)
// Split-K (grid.y) serves weight-gradient shapes whose tile count alone would leave CUs idle.
// Fused epilogue: bias, act' (GELU backward), dropout (counter-based mask), residual add, beta*C, second output
// (act / copy / dropout-masked copy), BatchNorm column statistics; fused A-row sums (bias gradients) from the
// A fragments in registers.
#pragma once
#include "common.h"

// The LDS-DMA inline asm writes M0 (declared as clobbered).  No compiler-generated code in these kernels uses M0
// (checked in the ISA: every M0 write is this asm's), so the "reserved register" warning is silenced here.
#pragma clang diagnostic ignored "-Winline-asm"

namespace awg {

constexpr int BN = 128;
constexpr int ROWB = 128;                // bytes of K per operand row per step (K-contiguous image pitch)
constexpr int CPITCH = BN + 4;           // f32 pitch of the epilogue tile

template <int BMT> struct Cfg;
#ifndef AW_W8
#define AW_W8 1
#endif
#if AW_W8
// 128-row tile, 8 waves of 32x64: 4 waves per SIMD at two workgroups per CU (MINB = min waves per SIMD)
template <> struct Cfg<128> { static constexpr int NTH = 512, NSTAGE = 2, MINB = 4; };
#else
template <> struct Cfg<128> { static constexpr int NTH = 256, NSTAGE = 2, MINB = 2; };
#endif
template <> struct Cfg<256> { static constexpr int NTH = 512, NSTAGE = 3, MINB = 1; };
template <int BMT> constexpr int stage_bytes() { return (BMT + BN) * ROWB; }
template <int BMT> constexpr int smem_bytes() {
  return Cfg<BMT>::NSTAGE * stage_bytes<BMT>() > BMT * CPITCH * 4 ? Cfg<BMT>::NSTAGE * stage_bytes<BMT>()
                                                                   : BMT * CPITCH * 4;
}

template <typename T> struct TT;
template <> struct TT<bf16> {
  static constexpr int EPC = 8, BK = 64;
  // rotation of k-row k (bytes): conflict-free ds_read_b64_tr_b16 for the 32-lane halves
  __device__ static constexpr int rot(int k) { return 32 * ((k & 3) + 4 * ((k >> 3) & 1)); }
};
template <> struct TT<float> {
  static constexpr int EPC = 4, BK = 32;
  __device__ static constexpr int rot(int k) { return 64 * ((k >> 2) & 1); }
};

// K-contiguous image [row][128 B]: logical 16-B chunk c of row r lives at physical chunk c ^ ((r >> 1) & 7)
// (conflict-free ds_read_b128 for the 16-row fragments; verified against the gfx950 lane groups).
__device__ __forceinline__ int nt_off(int row, int chunk) { return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4); }
// row-contiguous image [k][MPB bytes] (MPB = rows * sizeof(T)): byte b of k-row k lives at (b + rot(k)) mod MPB
template <typename T, int MPB>
__device__ __forceinline__ int tr_off(int krow, int byte_in_row) {
  return krow * MPB + ((byte_in_row + TT<T>::rot(krow)) & (MPB - 1));
}

struct GemmP {
  aw_gemm_args a;
  int tiles_n, nblocks, splits, ksplit;
  int vec;   // every epilogue operand row is 16-B aligned: vectorised epilogue
  int a_bytes, b_bytes;  // extents of A and B (buffer-descriptor ranges; < 2^31)
  float* ws; // split-K partial slabs [splits][M][N] (NULL: fp32 atomics)
  // grouped launch (aw_gemm_grouped): ngroups problems of one shape, tiles_per_group consecutive logical tiles
  // each; the operand / output / row-sum pointers of group g replace a.A, a.B, a.C, a.a_rowsum
  int ngroups, tiles_per_group;
  int bm;    // tile rows of this launch (128 or 256)
  const void* gA[AW_GEMM_MAX_GROUPS];
  const void* gB[AW_GEMM_MAX_GROUPS];
  void* gC[AW_GEMM_MAX_GROUPS];
  float* gRow[AW_GEMM_MAX_GROUPS];
};

enum { CONV_NONE = 0, CONV_ROWSHIFT = 1, CONV_KSHIFT = 2 };

// Epilogue codes: a specialised kernel is compiled per code in use (gemm_fast_*.hip); EP_GENERIC reads every
// feature from the argument block at run time (all other shapes / dtypes / alignments).
enum EpiBits : uint32_t {
  EP_BIAS = 1u << 0, EP_BIASMOD = 1u << 1, EP_PRE = 1u << 2, EP_TANH = 1u << 3, EP_DROP = 1u << 4,
  EP_RESID = 1u << 5, EP_BETA = 1u << 6, EP_C = 1u << 7, EP_CBF = 1u << 8, EP_C2ACT = 1u << 9,
  EP_C2COPY = 1u << 10, EP_C2DROP = 1u << 11, EP_C2BF = 1u << 12, EP_STATS = 1u << 13, EP_ACCUM = 1u << 14,
  EP_PREBF = 1u << 15, EP_RESIDBF = 1u << 16, EP_DERIV = 1u << 17, EP_C2DACT = 1u << 18, EP_GENERIC = 1u << 31
};

// Diagnostic phase stamps (tools/probe only: defined there before this file is included; never in the library).
#ifdef AW_GEMM_STAMPS
static __device__ uint64_t g_gemm_stamps[8192 * 8];   // one copy per translation unit (each has its own kernels)
#define AW_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 8192) \
    g_gemm_stamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// extern "C" reader of this translation unit's stamps (copies n words out, then zeroes them)
#define AW_STAMP_EXPORT(name)                                                                                   \
  extern "C" int name(uint64_t* out, int n) {                                                                  \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(awg::g_gemm_stamps), (size_t)n * 8) != hipSuccess) return -1;     \
    static uint64_t zeros[8192 * 8];                                                                            \
    return hipMemcpyToSymbol(HIP_SYMBOL(awg::g_gemm_stamps), zeros, sizeof(zeros)) == hipSuccess ? n : -1;    \
  }
#else
#define AW_STAMP(i) do { } while (0)
#define AW_STAMP_EXPORT(name)
#endif

// ---------------------------------------------------------------- operand staging
// Loads are raw buffer loads: an out-of-range byte offset returns zeros, which implements every mask
// (M/N/K tails, implicit-conv window edges) without branches.
constexpr int OOB = 0x7FFFFFF0;
typedef int v4i32 __attribute__((ext_vector_type(4)));

template <typename T, bool TR, int CONV, bool RAGGED, int ROWS, int NTH>
struct Stager {
  static constexpr int EPC = TT<T>::EPC, BK = TT<T>::BK;
  static constexpr int CPR = ROWS / EPC;            // 16-B chunks per k-row of a row-contiguous tile
  static constexpr int CPK = BK / EPC;              // chunks per row of a K-contiguous tile (8)
  static constexpr int MPB = ROWS * (int)sizeof(T); // bytes per k-row of the row-contiguous image
  static constexpr int NCH = ROWS * 8 / NTH;        // 16-B chunks per thread per step
  const T* base;
  int64_t ld;
  int rows_total, row0, kend, cin, seg, dir;
  __amdgpu_buffer_rsrc_t rsrc;
  v4i32 desc;       // the same buffer descriptor as four SGPR words (inline-asm LDS-DMA)
  // per-thread invariants of the implicit convolution (window position / tap of each chunk)
  int wpos[NCH];    // ROWSHIFT: row % seg (fixed rows);  KSHIFT: (k0 + krow) % seg, advanced per K step
  int tapoff[NCH];  // KSHIFT: row shift j-1 of the chunk's column tap
  int colin[NCH];   // KSHIFT: column within the tap (m - j*cin)

  // logical row offset (in elements) of chunk c of a row-contiguous image: register staging writes chunk c at
  // its logical place; LDS-DMA staging lands chunk c at physical byte 16*c, so it loads the logical chunk there
  __device__ __forceinline__ static int tr_logical_m(int c, bool dma) {
    if (!dma) return (c % CPR) * EPC;
    const int pb = (c % CPR) * 16;
    return ((pb - TT<T>::rot(c / CPR)) & (MPB - 1)) / (int)sizeof(T);
  }

  __device__ __forceinline__ void init(int kbeg, int tid, int nbytes, bool dma) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nbytes, 0x00020000);
    const uint64_t b = (uint64_t)(uintptr_t)base;
    desc = v4i32{(int)__builtin_amdgcn_readfirstlane((uint32_t)b),
                 (int)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu),
                 (int)__builtin_amdgcn_readfirstlane((uint32_t)nbytes), 0x00020000};
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NTH;
      if constexpr (CONV == CONV_ROWSHIFT) {
        wpos[i] = (row0 + c / CPK) % seg;
      } else if constexpr (CONV == CONV_KSHIFT) {
        const int m = row0 + tr_logical_m(c, dma);
        const int j = m / cin;
        tapoff[i] = j - 1;
        colin[i] = m - j * cin;
        wpos[i] = (kbeg + c / CPR) % seg;
      }
    }
  }

  __device__ __forceinline__ uint4 bload(int off) const {
    auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
    uint4 u;
    memcpy(&u, &r, 16);
    return u;
  }

  // source element index of the chunk at logical (row, k) of a K-contiguous tile; ok = not masked
  __device__ __forceinline__ int64_t src_nt(int i, int jrow, int row, int k, bool& ok) const {
    ok = row < rows_total && k < kend;
    int src = row, kk = k;
    if constexpr (CONV == CONV_ROWSHIFT) {
      kk = k - jrow * cin;
      const int sft = dir * (jrow - 1);
      ok = ok && (wpos[i] + sft >= 0) && (wpos[i] + sft < seg);
      src = row + sft;
    }
    return (int64_t)src * ld + kk;
  }
  // source element index of the chunk at logical (k, m) of a row-contiguous tile (KSHIFT advances its window)
  __device__ __forceinline__ int64_t src_tr(int i, int k, int m, bool& ok) {
    ok = k < kend && m < rows_total;
    int srck = k, mm = m;
    if constexpr (CONV == CONV_KSHIFT) {
      mm = colin[i];
      const int sft = tapoff[i];
      ok = ok && (wpos[i] + sft >= 0) && (wpos[i] + sft < seg);
      srck = k + sft;
      wpos[i] += BK % seg;                 // advance the window position to the next K step
      if (wpos[i] >= seg) wpos[i] -= seg;
    }
    return (int64_t)srck * ld + mm;
  }

  // register staging (ragged shapes): global -> VGPRs
  __device__ __forceinline__ void load(int k0, int tid, uint4 (&v)[NCH]) {
    // ROWSHIFT: cin % BK == 0, so the tap is uniform over the whole K step
    const int jrow = (CONV == CONV_ROWSHIFT) ? k0 / cin : 0;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NTH;
      bool ok;
      if constexpr (!TR) {
        const int k = k0 + (c % CPK) * EPC;
        const int64_t e = src_nt(i, jrow, row0 + c / CPK, k, ok);
        if constexpr (RAGGED) {
          if (ok && k + EPC > kend) {
            T tmp[EPC];
#pragma unroll
            for (int q = 0; q < EPC; ++q) tmp[q] = (k + q < kend) ? base[e + q] : from_f32<T>(0.f);
            memcpy(&v[i], tmp, 16);
            continue;
          }
        }
        v[i] = bload(ok ? (int)(e * (int)sizeof(T)) : OOB);
      } else {
        const int m = row0 + (c % CPR) * EPC;
        const int64_t e = src_tr(i, k0 + c / CPR, m, ok);
        if constexpr (RAGGED) {
          if (ok && m + EPC > rows_total) {
            T tmp[EPC];
#pragma unroll
            for (int q = 0; q < EPC; ++q) tmp[q] = (m + q < rows_total) ? base[e + q] : from_f32<T>(0.f);
            memcpy(&v[i], tmp, 16);
            continue;
          }
        }
        v[i] = bload(ok ? (int)(e * (int)sizeof(T)) : OOB);
      }
    }
  }

  __device__ __forceinline__ void store(char* lds, int tid, const uint4 (&v)[NCH]) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NTH;
      if constexpr (!TR)
        *reinterpret_cast<uint4*>(lds + nt_off(c / CPK, c % CPK)) = v[i];
      else
        *reinterpret_cast<uint4*>(lds + tr_off<T, MPB>(c / CPR, (c % CPR) * 16)) = v[i];
    }
  }

  // LDS-DMA staging (gfx950 buffer_load ... lds): chunk c = tid + i*NTH lands at byte 16*c of the operand's stage
  // image (lane-linear per wave instruction, base in M0); the swizzle is applied to the SOURCE address.
  // Issued from inline asm so that the compiler does not see an LDS write it cannot disambiguate from the ds_reads
  // of the other stages (it would drain vmcnt to 0 before every compute step and serialise the pipeline); the
  // kernel orders the DMA itself with counted vmcnt waits and barriers.
  // Everything that does not depend on the K step is computed once (dma_init): per step a chunk costs one add,
  // a few compares and a select; the step-dependent parts (tap shift, k0 * ld) are wave-uniform scalars.
  int doff[NCH];    // source byte offset of the chunk at K step 0 (current tap), OOB_F folded in where masked
  int rbase[NCH];   // ROWSHIFT: the unshifted, unmasked offset (doff is re-derived from it at every tap change)
  int dpos[NCH];    // logical k (K-contiguous image) or k-row (row-contiguous image) of the chunk within a step
  bool rok[NCH];    // the chunk's row (K-contiguous) / column block (row-contiguous) lies inside the operand
  uint32_t lds0;    // LDS byte address of this wave's first chunk in stage 0
  int dj, dkc;      // ROWSHIFT: tap and channel offset of the next K step (cin % BK == 0; steps issue in order)
  // A masked chunk carries OOB_F in its offset: OOB_F + any in-buffer delta (< 2^31) stays beyond num_records
  // (< 2^31) as an unsigned 32-bit offset, so the buffer load returns zeros without a per-step select.
  static constexpr uint32_t OOB_F = 0x80000000u;

  __device__ __forceinline__ void retap() {
    const int sft = dir * (dj - 1);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const bool ok = rok[i] && (unsigned)(wpos[i] + sft) < (unsigned)seg;
      doff[i] = ok ? rbase[i] + (int)((int64_t)sft * ld * (int)sizeof(T)) : (int)OOB_F;
    }
  }

  __device__ __forceinline__ void dma_init(int tid, uint32_t img_lds, int kbeg) {
    lds0 = img_lds + __builtin_amdgcn_readfirstlane((uint32_t)(tid & ~63)) * 16u;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NTH;
      if constexpr (!TR) {
        const int r = c / CPK;
        const int lc = (c % CPK) ^ ((r >> 1) & 7);
        const int row = row0 + r;
        rok[i] = row < rows_total;
        dpos[i] = lc * EPC;
        rbase[i] = rok[i] ? (int)(((int64_t)row * ld + lc * EPC) * (int)sizeof(T)) : 0;
        doff[i] = rok[i] ? rbase[i] : (int)OOB_F;
      } else {
        const int kr = c / CPR;
        const int m = row0 + tr_logical_m(c, true);
        rok[i] = m < rows_total;
        dpos[i] = kr;
        if constexpr (CONV == CONV_KSHIFT)
          doff[i] = (int)(((int64_t)(kr + tapoff[i]) * ld + colin[i]) * (int)sizeof(T));
        else
          doff[i] = rok[i] ? (int)(((int64_t)kr * ld + m) * (int)sizeof(T)) : (int)OOB_F;
      }
    }
    if constexpr (CONV == CONV_ROWSHIFT) {
      dj = kbeg / cin;
      dkc = kbeg - dj * cin;
      retap();
    }
  }

  // One K step's DMA.  Steps must be issued in increasing order, each once (ROWSHIFT keeps its tap state here).
  // Interior steps cost one add per chunk: row / tap masks are folded into doff, and the K-range test is only
  // evaluated on the (wave-uniform) partial last step.
  __device__ __forceinline__ void dma(int k0, uint32_t stage_off) {
    int delta;
    if constexpr (!TR)
      delta = (CONV == CONV_ROWSHIFT ? dkc : k0) * (int)sizeof(T);
    else
      delta = (int)((int64_t)k0 * ld * (int)sizeof(T));
    const bool full = k0 + BK <= kend;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int off;
      if constexpr (CONV == CONV_KSHIFT) {
        bool ok = rok[i] & (k0 + dpos[i] < kend);
        ok = ok & ((unsigned)(wpos[i] + tapoff[i]) < (unsigned)seg);
        wpos[i] += BK % seg;                 // advance the window position to the next K step
        if (wpos[i] >= seg) wpos[i] -= seg;
        off = ok ? doff[i] + delta : OOB;
      } else {
        off = doff[i] + delta;
        if (!full) off = (k0 + dpos[i] < kend) ? off : OOB;
      }
      const uint32_t m0 = lds0 + stage_off + (uint32_t)(i * NTH * 16);
      asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(desc)
                   : "memory", "m0");
    }
    if constexpr (CONV == CONV_ROWSHIFT) {
      dkc += BK;
      if (dkc >= cin) {
        dkc = 0;
        ++dj;
        retap();
      }
    }
  }
};

// ---------------------------------------------------------------- fragments
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// Fragment of the 16 rows [rbase, rbase+16) x this lane's K slice of MFMA sub-step u, as 16 bytes.
// K order inside a sub-step is the same for A and B: lane group g holds k = 8g..8g+7 (bf16) /
// k = 4g..4g+3 with one element per f32 MFMA (f32).
template <typename T, bool TR, int MPB>
__device__ __forceinline__ uint4 frag(const char* lds, int rbase, int lane, int u) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (!TR) {
    return *reinterpret_cast<const uint4*>(lds + nt_off(rbase + i, 4 * u + g));
  } else if constexpr (sizeof(T) == 2) {
    // two 4(k) x 16(row) transposed reads: lane 4q+p addresses k-row q, rows 4p..4p+3 of the block;
    // lane i receives row i, k-rows 0..3
    const int q = i >> 2, p = i & 3;
    const int k0 = 32 * u + 8 * g + q;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4i16*)(uintptr_t)(lds + tr_off<T, MPB>(k0, 2 * (rbase + 4 * p))));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4i16*)(uintptr_t)(lds + tr_off<T, MPB>(k0 + 4, 2 * (rbase + 4 * p))));
    uint4 out;
    memcpy(&out, &lo, 8);
    memcpy(reinterpret_cast<char*>(&out) + 8, &hi, 8);
    return out;
  } else {
    float f[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
      f[s] = *reinterpret_cast<const float*>(lds + tr_off<T, MPB>(16 * u + 4 * g + s, 4 * (rbase + i)));
    uint4 out;
    memcpy(&out, f, 16);
    return out;
  }
}

template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
  __device__ __forceinline__ static void run(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                  0, 0, 0);
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

// 4 consecutive elements (16-B aligned for f32, 8-B for bf16)
// Epilogue outputs are stored non-temporally: they are read back by a later launch (often the backward), never by
// this one, and allocating them in the XCD's L2 evicts the operand tiles the other workgroups are re-reading
// (A/B over the bench: VQ-VAE step -0.4 %, transformer step -2 %).
#ifndef AW_GEMM_NT
#define AW_GEMM_NT 1
#endif
// wt (aw_gemm_args.store_policy == AW_STORE_WT): write-through (sc1) stores instead -- the lines leave the XCD's L2
// at once, so the end-of-kernel release has no dirty output lines to write back before the next launch may start
// (the VQ-VAE step's chain of 64 class-A launches: +3 %, same-box A/B)
__device__ __forceinline__ void store4(void* base, bool is_bf16, int64_t e, const float (&v)[4], bool wt) {
  if (is_bf16) {
    bf16 h[4] = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    u32x2 u;
    memcpy(&u, h, 8);
    u32x2* d = reinterpret_cast<u32x2*>(reinterpret_cast<bf16*>(base) + e);
    if (wt) aw_st_wt(d, u);
    else if (AW_GEMM_NT) __builtin_nontemporal_store(u, d);
    else *d = u;
  } else {
    f32x4 u = {v[0], v[1], v[2], v[3]};
    f32x4* d = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(base) + e);
    if (wt) aw_st_wt(d, u);
    else if (AW_GEMM_NT) __builtin_nontemporal_store(u, d);
    else *d = u;
  }
}

// Bijective XCD-aware remap: consecutive logical tiles land on the same XCD (blocks b and b+8 share one).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = bid % 8, slot = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// sum of the K values one lane holds in an A fragment (8 bf16 or 4 f32)
template <typename T>
__device__ __forceinline__ float frag_sum(const uint4& v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (sizeof(T) == 2) {
    const bf16x8 h = __builtin_bit_cast(bf16x8, v);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0 += (float)h[2 * i];
      s1 += (float)h[2 * i + 1];
    }
    return s0 + s1;
  } else {
    return (__uint_as_float(w[0]) + __uint_as_float(w[1])) + (__uint_as_float(w[2]) + __uint_as_float(w[3]));
  }
}

template <int N> __device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <typename T, bool ATR, bool BTR, int ACONV, int BCONV, bool RAGGED, uint32_t EPI, int BMT>
__global__ __launch_bounds__(Cfg<BMT>::NTH, RAGGED ? 1 : Cfg<BMT>::MINB) void gemm_kernel(GemmP P) {
  constexpr int NTH = Cfg<BMT>::NTH;
  constexpr int BK = TT<T>::BK;
  constexpr int A_IMG = BMT * ROWB;                // A stage image bytes; the B image follows it
  constexpr int STAGE = stage_bytes<BMT>();
  static_assert(!(RAGGED && BMT != 128), "ragged shapes use the 128-row register-staged tile");
  using SA = Stager<T, ATR, ACONV, RAGGED, BMT, NTH>;
  using SB = Stager<T, BTR, BCONV, RAGGED, BN, NTH>;
  const aw_gemm_args& p = P.a;
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<BMT>()];

  AW_STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  constexpr int WR = BMT / (NTH / 128);            // rows per wave (waves form (NTH/128) x 2)
  constexpr int FM = WR / 16;                      // 16-row A fragments per wave
  int tile = xcd_remap(blockIdx.x, P.nblocks);
  const void* Aptr = p.A;
  const void* Bptr = p.B;
  void* Cptr = p.C;
  float* rowptr = p.a_rowsum;
  if (P.ngroups > 1) {   // consecutive logical tiles (one XCD) belong to one group: its operands share that L2
    const int g = tile / P.tiles_per_group;
    tile -= g * P.tiles_per_group;
    Aptr = P.gA[g];
    Bptr = P.gB[g];
    Cptr = P.gC[g];
    rowptr = P.gRow[g];
  }
  const int tm = tile / P.tiles_n, tn = tile % P.tiles_n;
  const int m0 = tm * BMT, n0 = tn * BN;
  const int M = p.M, N = p.N;
  const int kbeg = blockIdx.y * P.ksplit;
  const int kend = min(p.K, kbeg + P.ksplit);

  SA sa{reinterpret_cast<const T*>(Aptr), p.lda, M, m0, kend, p.conv_cin, p.conv_seg, p.conv_dir};
  SB sb{reinterpret_cast<const T*>(Bptr), p.ldb, N, n0, kend, p.conv_cin, p.conv_seg, 1};
  constexpr bool use_dma = !RAGGED;
  sa.init(kbeg, tid, P.a_bytes, use_dma);
  sb.init(kbeg, tid, P.b_bytes, use_dma);
  if constexpr (use_dma) {
    const uint32_t smem_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    sa.dma_init(tid, smem_lds, kbeg);
    sb.dma_init(tid, smem_lds + A_IMG, kbeg);
  }
  const bool do_rowsum = rowptr != nullptr && tn == 0;

  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused A-row sums (bias gradients) from the A fragments already in registers: waves wn == 0 of the tn == 0
  // tiles add their 8 (bf16) / 4 (f32) k-values per fragment; the lane groups are reduced once at the end
  constexpr bool ROWSUM_OK = (EPI & EP_GENERIC) || (EPI & EP_ACCUM);   // bias gradients: weight-gradient launches
  const bool wave_rowsum = ROWSUM_OK && do_rowsum && wn == 0;
  float rowacc[FM] = {};

  auto compute = [&](const char* a_l) {
    const char* b_l = a_l + A_IMG;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint4 af[FM], bfr[4];
#pragma unroll
      for (int f = 0; f < FM; ++f) af[f] = frag<T, ATR, BMT * (int)sizeof(T)>(a_l, wm * WR + f * 16, lane, u);
#pragma unroll
      for (int f = 0; f < 4; ++f) bfr[f] = frag<T, BTR, BN * (int)sizeof(T)>(b_l, wn * 64 + f * 16, lane, u);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Mfma<T>::run(acc[i][j], af[i], bfr[j]);
      if (wave_rowsum) {
#pragma unroll
        for (int f = 0; f < FM; ++f) rowacc[f] += frag_sum<T>(af[f]);
      }
    }
  };

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if constexpr (use_dma && Cfg<BMT>::NSTAGE == 2) {
    // two stages: the loads of step t+1 fly into the other stage while step t computes
    char* L0 = smem;
    char* L1 = smem + STAGE;
    sa.dma(kbeg, 0u);
    sb.dma(kbeg, 0u);
    wait_vmcnt<0>();
    __syncthreads();
    AW_STAMP(1);
    for (int kt = 0; kt < nk; ++kt) {
      char* cur = (kt & 1) ? L1 : L0;
      const uint32_t nxt = (kt & 1) ? 0u : (uint32_t)STAGE;
      if (kt + 1 < nk) {
        sa.dma(kbeg + (kt + 1) * BK, nxt);
        sb.dma(kbeg + (kt + 1) * BK, nxt);
      }
      compute(cur);
      wait_vmcnt<0>();
      __syncthreads();
    }
  } else if constexpr (use_dma) {
    // 256-row tile, one workgroup per CU: two wave groups ping-pong (the 8-wave schedule of the guide, as in
    // wgrad.hip).  Group g = waves 4g..4g+3 (rows 128g..128g+127, one wave per SIMD); group 1 runs one barrier
    // behind group 0, so on every SIMD one wave issues its fragment reads (16 ds_read_b128 / tr pairs) and the DMA
    // of step t + 2 while its partner runs 32 MFMAs.  Three LDS stages: the DMA of step t + 2 overwrites the stage
    // of step t - 1, whose reads both groups retired before the last barrier (lgkmcnt(0) ending each read segment);
    // each wave retires its own DMA of step t + 1 with a counted vmcnt, the barrier publishes it.
    constexpr int PER_STEP = SA::NCH + SB::NCH;
    const int grp = wid >> 2;
    auto stage_of = [](int t) { return (uint32_t)((t % 3) * STAGE); };
    sa.dma(kbeg, 0u);
    sb.dma(kbeg, 0u);
    if (nk > 1) {
      sa.dma(kbeg + BK, stage_of(1));
      sb.dma(kbeg + BK, stage_of(1));
      wait_vmcnt<PER_STEP>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (grp == 1) __builtin_amdgcn_s_barrier();
    AW_STAMP(1);
    uint4 af[2][FM], bfr[2][4];
    for (int kt = 0; kt < nk; ++kt) {
      const char* a_l = smem + stage_of(kt);
      const char* b_l = a_l + A_IMG;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int f = 0; f < FM; ++f) af[u][f] = frag<T, ATR, BMT * (int)sizeof(T)>(a_l, wm * WR + f * 16, lane, u);
#pragma unroll
        for (int f = 0; f < 4; ++f) bfr[u][f] = frag<T, BTR, BN * (int)sizeof(T)>(b_l, wn * 64 + f * 16, lane, u);
      }
      if (kt + 2 < nk) {
        sa.dma(kbeg + (kt + 2) * BK, stage_of(kt + 2));
        sb.dma(kbeg + (kt + 2) * BK, stage_of(kt + 2));
        wait_vmcnt<PER_STEP>();            // step kt + 1 retired, kt + 2 in flight
      } else {
        wait_vmcnt<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) Mfma<T>::run(acc[i][j], af[u][i], bfr[u][j]);
      __builtin_amdgcn_s_setprio(0);
      if (wave_rowsum) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int f = 0; f < FM; ++f) rowacc[f] += frag_sum<T>(af[u][f]);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();   // both groups end on the same barrier count
  } else {
    // register staging (ragged shapes): LDS stage s holds K step t (t % 2 == s) while the registers of the other
    // set carry the loads of step t+1; the loads of step t+2 are issued at the top of step t
    char* L0 = smem;
    char* L1 = smem + STAGE;
    uint4 ra0[SA::NCH], rb0[SB::NCH], ra1[SA::NCH], rb1[SB::NCH];
    sa.load(kbeg, tid, ra0);
    sb.load(kbeg, tid, rb0);
    sa.load(kbeg + BK, tid, ra1);
    sb.load(kbeg + BK, tid, rb1);
    sa.store(L0, tid, ra0);
    sb.store(L0 + A_IMG, tid, rb0);
    __syncthreads();
    AW_STAMP(1);
    for (int kt = 0; kt < nk; kt += 2) {
      sa.load(kbeg + (kt + 2) * BK, tid, ra0);   // beyond kend: out-of-range -> zeros, never read
      sb.load(kbeg + (kt + 2) * BK, tid, rb0);
      compute(L0);
      sa.store(L1, tid, ra1);
      sb.store(L1 + A_IMG, tid, rb1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      sa.load(kbeg + (kt + 3) * BK, tid, ra1);
      sb.load(kbeg + (kt + 3) * BK, tid, rb1);
      compute(L1);
      sa.store(L0, tid, ra0);
      sb.store(L0 + A_IMG, tid, rb0);
      __syncthreads();
    }
  }

  AW_STAMP(2);
  if (wave_rowsum) {
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      float v = rowacc[f];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int r = m0 + wm * WR + f * 16 + lane;
      if (lane < 16 && r < M) atomicAdd(rowptr + r, v);
    }
  }

  // ---------------------------------------------------------------- epilogue
  // Every feature test below is a compile-time constant for a specialised EPI code (see EpiBits) and a runtime
  // test of the argument block for EP_GENERIC, so each hot epilogue compiles to straight-line code.
#define EPF(bit, rt) ((EPI & EP_GENERIC) ? (rt) : ((EPI & (bit)) != 0))
  constexpr bool GEN = (EPI & EP_GENERIC) != 0;
  constexpr int NR = NTH / 32;                     // rows per pass of the row-major epilogue walk
  // 1) accumulators -> LDS tile (static register indexing), 2) one element per thread per step with
  //    consecutive threads on consecutive columns: every wave instruction touches 256 contiguous bytes.
  float* Cs = reinterpret_cast<float*>(smem);
  {
    const int cq = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(wm * WR + i * 16 + rq + r) * CPITCH + wn * 64 + j * 16 + cq] = acc[i][j][r];
  }
  __syncthreads();
  AW_STAMP(3);
  const int rows_here = min(BMT, M - m0);
  if (EPF(EP_ACCUM, P.splits > 1 || p.accumulate)) {
    if (P.splits > 1 && P.ws) {  // partial slab of this split: plain coalesced stores, reduced by gemm_reduce
      const int lc = tid & 127, col = n0 + lc;
      if (col >= N) return;
      float* slab = P.ws + (int64_t)blockIdx.y * M * N;
      for (int lr = tid >> 7; lr < rows_here; lr += NTH / 128)
        slab[(int64_t)(m0 + lr) * N + col] = Cs[lr * CPITCH + lc];
      return;
    }
    // accumulate into f32 C with atomics (consecutive lanes -> columns)
    const int lc = tid & 127, col = n0 + lc;
    if (col >= N) return;
    const int64_t oc = p.col_mod > 0 ? (int64_t)(col % p.col_mod) * p.col_mul + col / p.col_mod + p.col_off
                                     : (int64_t)col * (p.col_mul > 0 ? p.col_mul : 1) + p.col_off;
    float* C = reinterpret_cast<float*>(Cptr);
    for (int lr = tid >> 7; lr < rows_here; lr += NTH / 128)
      atomicAdd(C + (int64_t)(m0 + lr) * p.ldc + oc, p.alpha * Cs[lr * CPITCH + lc]);
    return;
  }
  if constexpr (!GEN && (EPI & EP_ACCUM)) return;
  else {
  const bool f_bias = EPF(EP_BIAS, p.bias != nullptr);
  const bool f_bmod = EPF(EP_BIASMOD, p.bias_mod > 0);
  const bool f_pre = EPF(EP_PRE, p.pre != nullptr);
  const bool f_prebf = EPF(EP_PREBF, p.pre_dtype == AW_BF16);
  const bool f_tanh = EPF(EP_TANH, p.act == AW_ACT_GELU_TANH);
  const bool f_deriv = EPF(EP_DERIV, p.act == AW_ACT_DERIV);   // pre holds act' itself
  const bool f_drop = EPF(EP_DROP, p.drop_p > 0.f);
  const bool f_resid = EPF(EP_RESID, p.resid != nullptr);
  const bool f_residbf = EPF(EP_RESIDBF, p.resid_dtype == AW_BF16);
  const bool f_beta = EPF(EP_BETA, p.beta != 0.f);
  const bool f_c = EPF(EP_C, Cptr != nullptr);
  const bool f_cbf = EPF(EP_CBF, p.c_dtype == AW_BF16);
  const int c2m = GEN ? p.c2_mode
                      : ((EPI & EP_C2ACT) ? 1 : (EPI & EP_C2COPY) ? 2 : (EPI & EP_C2DROP) ? 3 : (EPI & EP_C2DACT) ? 4 : 0);
  const bool f_c2bf = EPF(EP_C2BF, p.c2_dtype == AW_BF16);
  const bool f_stats = EPF(EP_STATS, p.colstats != nullptr);
  const float alpha = GEN ? p.alpha : 1.f;       // specialised codes are issued for alpha == 1 only
  const bool wt = p.store_policy == AW_STORE_WT;
  constexpr bool FASTGELU = sizeof(T) == 2;      // bf16 operands: branch-free erf (exact-f32 mode keeps erff)
  const uint64_t dseed = f_drop ? aw_seed_mix(p.drop_seed, p.seed_ptr) : 0ull;
  const uint64_t dseed2 = c2m == 3 ? aw_seed_mix(p.drop2_seed, p.seed_ptr) : 0ull;
  // thread -> 4 consecutive columns (c4) x rows r0, r0+NR, ...; 4 rows of loads in flight per thread
  const int c4 = (tid & 31) * 4, r0 = tid >> 5;
  const int col = n0 + c4;
  // specialised codes are issued only when every operand row is 16-B aligned and N % 4 == 0
  const bool vec = GEN ? (P.vec && col + 4 <= N) : (col < N);
  float bias[4], csum[4] = {0.f, 0.f, 0.f, 0.f}, csq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = col + e;
    bias[e] = (f_bias && c < N) ? p.bias[f_bmod ? c % p.bias_mod : c] : 0.f;
  }
  if (col < N) {
    for (int lr0 = r0; lr0 < rows_here; lr0 += 4 * NR) {
      float4 pre4[4], res4[4], old4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // issue the operand loads of 4 rows first
        const int lr = lr0 + NR * u;
        if (lr >= rows_here) break;
        const int64_t row = m0 + lr;
        if (vec) {
          if (f_pre) {
            if (f_prebf) {
              const uint2 h = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(p.pre) + row * p.ld_pre + col);
              pre4[u] = make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xFFFF0000u),
                                    __uint_as_float(h.y << 16), __uint_as_float(h.y & 0xFFFF0000u));
            } else {
              pre4[u] = *reinterpret_cast<const float4*>(p.pre + row * p.ld_pre + col);
            }
          }
          if (f_resid) {
            if (f_residbf) {
              const uint2 h = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(p.resid) + row * p.ld_resid + col);
              res4[u] = make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xFFFF0000u),
                                    __uint_as_float(h.y << 16), __uint_as_float(h.y & 0xFFFF0000u));
            } else {
              res4[u] = *reinterpret_cast<const float4*>(p.resid + row * p.ld_resid + col);
            }
          }
          if (f_beta) old4[u] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Cptr) + row * p.ldc + col);
        } else if constexpr (GEN) {
          float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f}, c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (col + e >= N) break;
            if (f_pre) a[e] = load_as_f32(p.pre, p.pre_dtype, row * p.ld_pre + col + e);
            if (f_resid) b[e] = load_as_f32(p.resid, p.resid_dtype, row * p.ld_resid + col + e);
            if (f_beta) c[e] = reinterpret_cast<const float*>(Cptr)[row * p.ldc + col + e];
          }
          pre4[u] = make_float4(a[0], a[1], a[2], a[3]);
          res4[u] = make_float4(b[0], b[1], b[2], b[3]);
          old4[u] = make_float4(c[0], c[1], c[2], c[3]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int lr = lr0 + NR * u;
        if (lr >= rows_here) break;
        const int64_t row = m0 + lr;
        const float4 a4 = *reinterpret_cast<const float4*>(Cs + lr * CPITCH + c4);
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
        const float pv[4] = {pre4[u].x, pre4[u].y, pre4[u].z, pre4[u].w};
        const float rv[4] = {res4[u].x, res4[u].y, res4[u].z, res4[u].w};
        const float ov[4] = {old4[u].x, old4[u].y, old4[u].z, old4[u].w};
        const uint64_t e0 = (uint64_t)row * N + col;
        float ds[4] = {1.f, 1.f, 1.f, 1.f}, ds2[4] = {1.f, 1.f, 1.f, 1.f};
        if (f_drop) aw_dropout_scale4(dseed, e0, p.drop_p, ds);
        if (c2m == 3) aw_dropout_scale4(dseed2, e0, p.drop2_p, ds2);
        float v[4], w[4], ag[4];
        // bf16 operands: GELU and GELU' in packed pairs (aw_gelu4 / aw_gelu_grad4, shared with the encoder chain)
        if (FASTGELU && f_pre && !f_tanh && !f_deriv) aw_gelu_grad4(pv, ag);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = alpha * av[e] + bias[e];
          // x * act' * ds + resid with the last multiply fused into the add (aw_epi_mad): one rounding order that the
          // encoder chain (reschain.hip) reproduces exactly, whatever FMA contraction the compiler would choose
          float m = 1.f;
          bool has_m = false;
          if (f_pre) {
            const float a = f_deriv ? pv[e] : f_tanh ? gelu_tanh_grad(pv[e]) : (FASTGELU ? ag[e] : gelu_erf_grad(pv[e]));
            if (f_drop) x *= a;
            else m = a, has_m = true;
          }
          if (f_drop) m = ds[e], has_m = true;
          x = aw_epi_mad(x, m, has_m, f_resid ? rv[e] : 0.f, f_resid);
          if (f_beta) x += p.beta * ov[e];
          v[e] = x;
          float y = x;
          if (c2m == 1 && (f_tanh || !FASTGELU)) y = f_tanh ? gelu_tanh(x) : gelu_erf(x);
          else if (c2m == 3) y = x * ds2[e];
          w[e] = y;
          if (f_stats && col + e < N) {
            csum[e] += x;
            csq[e] += x * x;
          }
        }
        if (FASTGELU && c2m == 1 && !f_tanh) aw_gelu4(v, w);
        if (c2m == 4 && f_tanh && FASTGELU) {   // C = act(v), C2 = act'(v) from one exponential, packed pairs
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            f32x2 g, dg;
            gelu_tanh_and_grad2((f32x2){v[e], v[e + 1]}, g, dg);
            v[e] = g.x, v[e + 1] = g.y, w[e] = dg.x, w[e + 1] = dg.y;
          }
        } else if (c2m == 4) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float g, dg;
            if (f_tanh) {
              gelu_tanh_and_grad(v[e], g, dg);
            } else {
              float ex;
              const float phi = FASTGELU ? aw_phi_e(v[e], ex) : 0.f;
              g = FASTGELU ? v[e] * phi : gelu_erf(v[e]);
              dg = FASTGELU ? fmaf(v[e] * AW_INV_SQRT2PI, ex, phi) : gelu_erf_grad(v[e]);
            }
            v[e] = g;
            w[e] = dg;
          }
        }
        if (vec) {
          if (f_c) store4(Cptr, f_cbf, row * p.ldc + col, v, wt);
          if (c2m) store4(p.C2, f_c2bf, row * p.ldc2 + col, w, wt);
        } else if constexpr (GEN) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (col + e >= N) break;
            if (f_c) store_from_f32(Cptr, p.c_dtype, row * p.ldc + col + e, v[e]);
            if (c2m) store_from_f32(p.C2, p.c2_dtype, row * p.ldc2 + col + e, w[e]);
          }
        }
      }
    }
  }
  AW_STAMP(4);
  if (f_stats) {  // BatchNorm batch statistics: reduce the NR row-groups of a column, one f64 atomic each
    __syncthreads();
    float* red = Cs;   // [NR][2][128]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[(r0 * 2 + 0) * 128 + c4 + e] = csum[e];
      red[(r0 * 2 + 1) * 128 + c4 + e] = csq[e];
    }
    __syncthreads();
    if (tid < 128 && n0 + tid < N) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int g = 0; g < NR; ++g) {
        a += red[(g * 2 + 0) * 128 + tid];
        b += red[(g * 2 + 1) * 128 + tid];
      }
      const int sl = (n0 + tid) % p.stats_mod;
      atomicAdd(p.colstats + sl, (double)a);
      atomicAdd(p.colstats + p.stats_mod + sl, (double)b);
    }
  }
  }
#undef EPF
}

// operand-layout variants of the kernel
enum Layout { L_NN = 0, L_NN_CONV = 1, L_NT = 2, L_NT_CONV = 3, L_TN = 4, L_TT = 5, L_TT_KCONV = 6 };

template <Layout LY> struct LayoutArgs;
template <> struct LayoutArgs<L_NN> { static constexpr bool ATR = false, BTR = false; static constexpr int AC = CONV_NONE, BC = CONV_NONE; };
template <> struct LayoutArgs<L_NN_CONV> { static constexpr bool ATR = false, BTR = false; static constexpr int AC = CONV_ROWSHIFT, BC = CONV_NONE; };
template <> struct LayoutArgs<L_NT> { static constexpr bool ATR = false, BTR = true; static constexpr int AC = CONV_NONE, BC = CONV_NONE; };
template <> struct LayoutArgs<L_NT_CONV> { static constexpr bool ATR = false, BTR = true; static constexpr int AC = CONV_ROWSHIFT, BC = CONV_NONE; };
template <> struct LayoutArgs<L_TN> { static constexpr bool ATR = true, BTR = false; static constexpr int AC = CONV_NONE, BC = CONV_NONE; };
template <> struct LayoutArgs<L_TT> { static constexpr bool ATR = true, BTR = true; static constexpr int AC = CONV_NONE, BC = CONV_NONE; };
template <> struct LayoutArgs<L_TT_KCONV> { static constexpr bool ATR = true, BTR = true; static constexpr int AC = CONV_NONE, BC = CONV_KSHIFT; };

template <typename T, Layout LY, bool RAGGED, uint32_t EPI, int BMT>
inline void launch_kernel(const GemmP& P, hipStream_t s) {
  using LA = LayoutArgs<LY>;
  hipLaunchKernelGGL((gemm_kernel<T, LA::ATR, LA::BTR, LA::AC, LA::BC, RAGGED, EPI, BMT>), dim3(P.nblocks, P.splits),
                     dim3(Cfg<BMT>::NTH), 0, s, P);
}

// non-ragged launch with the tile the host chose (P.bm; the 256-row tile exists for the generic and accumulate
// epilogues only -- the host issues specialised codes with 128-row tiles)
template <typename T, Layout LY, uint32_t EPI>
inline void launch_tiled(const GemmP& P, hipStream_t s) {
  if constexpr (sizeof(T) == 2 && (EPI == EP_GENERIC || EPI == EP_ACCUM)) {
    if (P.bm == 256) {
      launch_kernel<T, LY, false, EPI, 256>(P, s);
      return;
    }
  }
  launch_kernel<T, LY, false, EPI, 128>(P, s);
}

// Specialised-epilogue launchers (gemm_fast_fwd.hip, gemm_fast_bwd.hip): return false when (dtype, layout,
// code) has no compiled specialisation, so the caller falls back to the EP_GENERIC kernel.
bool launch_fast_fwd(const GemmP& P, hipStream_t s, bool is_bf16, Layout ly, uint32_t code);
bool launch_fast_bwd(const GemmP& P, hipStream_t s, bool is_bf16, Layout ly, uint32_t code);
bool launch_fast_256(const GemmP& P, hipStream_t s, Layout ly, uint32_t code);   // bf16, P.bm == 256
// The grouped decoder k = 3 weight gradient on the 8-wave ping-pong kernel (wgrad.hip); false when the shape or
// the policy (aw_gemm_set_wgrad_policy) rules it out (the caller then runs the generic grouped GEMM).
bool wgrad_conv3_try(const aw_gemm_args* args, int n, hipStream_t s);


}  // namespace awg
