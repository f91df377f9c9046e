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

constexpr int kMaxT = W2V_NV <= 16 ? 8 : 4;  // d > 1024: 4 target rows per batch

// wide: CBOW with 2 * window + 1 > 64 (skip-gram takes any window in one kernel)
KernelFn W2V_CAT(pick_train_nv, W2V_NV)(bool cbow, bool hs, bool ns, bool replay, bool wide) {
#define W2V_K(CB, H, N, R, WD) &train_epoch_kernel<W2V_NV, kMaxT, CB, H, N, R, WD>
#define W2V_KR(CB, H, N, WD) (replay ? W2V_K(CB, H, N, true, WD) : W2V_K(CB, H, N, false, WD))
#define W2V_KW(H, N) (wide ? W2V_KR(true, H, N, true) : W2V_KR(true, H, N, false))
  if (cbow) {
    if (hs && ns) return W2V_KW(true, true);
    if (hs) return W2V_KW(true, false);
    return W2V_KW(false, true);
  }
  if (hs && ns) return W2V_KR(false, true, true, false);
  if (hs) return W2V_KR(false, true, false, false);
  return W2V_KR(false, false, true, false);
#undef W2V_KW
#undef W2V_KR
#undef W2V_K
}

// hierarchical softmax without negatives (the large-vocabulary HS policy's
// capped launches): the low-occupancy, deep-pipeline kernel
KernelFn W2V_CAT(pick_train_deep_nv, W2V_NV)(bool cbow) {
  constexpr int M = kDeepMaxT<W2V_NV>;
  return cbow ? &train_epoch_deep_kernel<W2V_NV, M, true, true, false, false, false>
              : &train_epoch_deep_kernel<W2V_NV, M, false, true, false, false, false>;
}

ApplyFn W2V_CAT(pick_apply_nv, W2V_NV)() { return &apply_rows_kernel<W2V_NV>; }

}  // namespace w2v
