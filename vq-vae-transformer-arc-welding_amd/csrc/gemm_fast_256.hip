// Specialised-epilogue instantiations on the 256-row ping-pong tile (gemm_core.h main loop, one workgroup per CU)
// for the bf16 forward and input-gradient layouts: the class-A launches of the ResBlock stacks and the transformer
// (M = tokens, N = 512 .. 2048) when 256-row tiles fill the chip (gemm.hip: plan).
#include "gemm_fast_codes.h"

namespace awg {

#define AW_FAST_CASE256(T, LY, CODE) \
  case (CODE): launch_kernel<T, LY, false, (CODE), 256>(P, s); return true;

bool launch_fast_256(const GemmP& P, hipStream_t s, Layout ly, uint32_t code) {
  switch (ly) {
    case L_NN:
      switch (code) {
        AW_FWD_CODES(AW_FAST_CASE256, bf16, L_NN)
        AW_FWD_PLAIN_CODES(AW_FAST_CASE256, bf16, L_NN)
        default: return false;
      }
    case L_NN_CONV:
      switch (code) {
        AW_FWD_CODES(AW_FAST_CASE256, bf16, L_NN_CONV)
        default: return false;
      }
    case L_NT:
      switch (code) {
        AW_BWD_CONV_CODES(AW_FAST_CASE256, bf16, L_NT)
        AW_BWD_PLAIN_CODES(AW_FAST_CASE256, bf16, L_NT)
        default: return false;
      }
    case L_NT_CONV:
      switch (code) {
        AW_BWD_CONV_CODES(AW_FAST_CASE256, bf16, L_NT_CONV)
        default: return false;
      }
    default:
      return false;
  }
}

}  // namespace awg

AW_STAMP_EXPORT(aw_probe_stamps_256)   // probe builds only (AW_GEMM_STAMPS)
