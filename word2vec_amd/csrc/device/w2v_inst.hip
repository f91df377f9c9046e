// One row width's kernel instantiations (built once per W2V_NV by the
// Makefile so the 9 widths compile in parallel); w2v_dev.hip dispatches.
#include "w2v_kernels.hpp"
#include "w2v_launch.hpp"

#ifndef W2V_NV
#error "build with -DW2V_NV=<floats per lane>"
#endif

#define W2V_CAT2(a, b) a##b
#define W2V_CAT(a, b) W2V_CAT2(a, b)

namespace w2v {

constexpr int kMaxT = 8;

KernelFn W2V_CAT(pick_train_nv, W2V_NV)(bool cbow, bool hs, bool ns, bool replay) {
#define W2V_K(CB, H, N, R) &train_epoch_kernel<W2V_NV, kMaxT, CB, H, N, R>
#define W2V_KR(CB, H, N) (replay ? W2V_K(CB, H, N, true) : W2V_K(CB, H, N, false))
  if (cbow) {
    if (hs && ns) return W2V_KR(true, true, true);
    if (hs) return W2V_KR(true, true, false);
    return W2V_KR(true, false, true);
  }
  if (hs && ns) return W2V_KR(false, true, true);
  if (hs) return W2V_KR(false, true, false);
  return W2V_KR(false, false, true);
#undef W2V_KR
#undef W2V_K
}

ApplyFn W2V_CAT(pick_apply_nv, W2V_NV)() { return &apply_rows_kernel<W2V_NV>; }

}  // namespace w2v
