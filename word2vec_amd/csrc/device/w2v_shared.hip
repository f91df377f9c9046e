// Instantiations of the shared-negatives minibatch kernel (w2v_shared.hpp),
// one per row pitch of 64 KB floats; w2v_dev.hip dispatches.
#include "w2v_launch.hpp"
#include "w2v_shared.hpp"

namespace w2v {

KernelFn pick_shared_neg(int kb) {
  switch (kb) {
    case 1: return &train_shared_neg_kernel<1>;
    case 2: return &train_shared_neg_kernel<2>;
    case 3: return &train_shared_neg_kernel<3>;
    case 4: return &train_shared_neg_kernel<4>;
    case 5: return &train_shared_neg_kernel<5>;
    case 6: return &train_shared_neg_kernel<6>;
    case 7: return &train_shared_neg_kernel<7>;
    case 8: return &train_shared_neg_kernel<8>;
    case 10: return &train_shared_neg_kernel<10>;
    case 12: return &train_shared_neg_kernel<12>;
    case 16: return &train_shared_neg_kernel<16>;
    default: return nullptr;
  }
}

}  // namespace w2v
