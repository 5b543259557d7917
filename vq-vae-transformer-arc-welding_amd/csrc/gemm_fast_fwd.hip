// Specialised-epilogue instantiations of the MFMA GEMM for the forward layouts, 128-row tiles (codes:
// gemm_fast_codes.h; the 256-row ping-pong forms are in gemm_fast_256.hip).
#include "gemm_fast_codes.h"

namespace awg {

#define AW_FAST_CASE128(T, LY, CODE) \
  case (CODE): launch_kernel<T, LY, false, (CODE), 128>(P, s); return true;

bool launch_fast_fwd(const GemmP& P, hipStream_t s, bool is_bf16, Layout ly, uint32_t code) {
  if (P.bm == 256) return is_bf16 && launch_fast_256(P, s, ly, code);
  if (is_bf16 && ly == L_NN) {
    switch (code) {
      AW_FWD_CODES(AW_FAST_CASE128, bf16, L_NN)
      AW_FWD_PLAIN_CODES(AW_FAST_CASE128, bf16, L_NN)
      default: return false;
    }
  }
  if (is_bf16 && ly == L_NN_CONV) {
    switch (code) {
      AW_FWD_CODES(AW_FAST_CASE128, bf16, L_NN_CONV)
      default: return false;
    }
  }
  if (!is_bf16 && ly == L_NN) {
    switch (code) {
      AW_FWD_F32_CODES(AW_FAST_CASE128, float, L_NN)
      default: return false;
    }
  }
  return false;
}

}  // namespace awg

AW_STAMP_EXPORT(aw_probe_stamps_fwd)   // probe builds only (AW_GEMM_STAMPS)
