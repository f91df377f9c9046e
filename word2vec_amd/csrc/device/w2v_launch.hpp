// Kernel entry points per row width (defined in w2v_inst.hip, one object per width).
#pragma once
#include <stdint.h>

namespace w2v {

struct TrainArgs;
using KernelFn = void (*)(TrainArgs);
using ApplyFn = void (*)(float*, int64_t, int, const float*, float*, const uint8_t*, int, float, int);

#define W2V_DECLARE_NV(N)                                            \
  KernelFn pick_train_nv##N(bool cbow, bool hs, bool ns, bool replay, bool wide); \
  KernelFn pick_train_deep_nv##N(bool cbow); \
  ApplyFn pick_apply_nv##N();
W2V_DECLARE_NV(1)
W2V_DECLARE_NV(2)
W2V_DECLARE_NV(3)
W2V_DECLARE_NV(4)
W2V_DECLARE_NV(5)
W2V_DECLARE_NV(6)
W2V_DECLARE_NV(8)
W2V_DECLARE_NV(12)
W2V_DECLARE_NV(16)
W2V_DECLARE_NV(24)
W2V_DECLARE_NV(32)
#undef W2V_DECLARE_NV

// Shared-negatives minibatch SG (w2v_shared.hip) for a row pitch (floats, a
// multiple of 64 up to 1024, not 576/704/832/960); *waves = wavefronts per
// workgroup; occ = register budget in waves per SIMD (3; else the
// compiler's choice). Null for a pitch without an instantiation.
KernelFn pick_shared_neg(int64_t pitch, int occ, int* waves);

}  // namespace w2v
