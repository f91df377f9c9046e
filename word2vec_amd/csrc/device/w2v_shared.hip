// Instantiations of the shared-negatives minibatch kernel (w2v_shared.hpp):
// the row pitch decides the waves per center (2 up to 512 floats, 4 beyond)
// and the 16-column blocks per wave; w2v_dev.hip dispatches. (d512 over 4
// waves of 8 blocks, LDS-limited to 2 workgroups per CU: 62.3 vs 67.8 M
// words/s on configs[4].)
#include "w2v_launch.hpp"
#include "w2v_shared.hpp"

namespace w2v {

template <int KB, int NW>
static KernelFn pick_occ(int) {
  return &train_shared_neg_kernel<KB, NW, 2>;
}

KernelFn pick_shared_neg(int64_t pitch, int occ, int* waves) {
  if (pitch % 64 != 0) return nullptr;
  *waves = pitch <= 512 ? 2 : 4;
  switch (pitch / 64) {
    case 1: return pick_occ<2, 2>(occ);
    case 2: return pick_occ<4, 2>(occ);
    case 3: return pick_occ<6, 2>(occ);
    case 4: return pick_occ<8, 2>(occ);
    case 5: return pick_occ<10, 2>(occ);
    case 6: return pick_occ<12, 2>(occ);
    case 7: return pick_occ<14, 2>(occ);
    case 8: return pick_occ<16, 2>(occ);
    case 10: return pick_occ<10, 4>(occ);
    case 12: return pick_occ<12, 4>(occ);
    case 14: return pick_occ<14, 4>(occ);
    case 16: return pick_occ<16, 4>(occ);
    default: return nullptr;
  }
}

}  // namespace w2v
