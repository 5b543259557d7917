// Specialised-epilogue instantiations of the MFMA GEMM for the input-gradient layouts, 128-row tiles (codes:
// gemm_fast_codes.h; the 256-row ping-pong forms are in gemm_fast_256.hip).
#include "gemm_fast_codes.h"

namespace awg {

#define AW_FAST_CASE128(T, LY, CODE) \
  case (CODE): launch_kernel<T, LY, false, (CODE), 128>(P, s); return true;

bool launch_fast_bwd(const GemmP& P, hipStream_t s, bool is_bf16, Layout ly, uint32_t code) {
  if (P.bm == 256) return is_bf16 && launch_fast_256(P, s, ly, code);
  if (is_bf16 && ly == L_NT) {
    switch (code) {
      AW_BWD_CONV_CODES(AW_FAST_CASE128, bf16, L_NT)
      AW_BWD_PLAIN_CODES(AW_FAST_CASE128, bf16, L_NT)
      default: return false;
    }
  }
  if (is_bf16 && ly == L_NT_CONV) {
    switch (code) {
      AW_BWD_CONV_CODES(AW_FAST_CASE128, bf16, L_NT_CONV)
      default: return false;
    }
  }
  return false;
}

}  // namespace awg

AW_STAMP_EXPORT(aw_probe_stamps_bwd)   // probe builds only (AW_GEMM_STAMPS)
