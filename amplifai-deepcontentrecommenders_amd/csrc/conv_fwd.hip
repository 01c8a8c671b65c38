// Forward convolutions of the item tower (k_conv_rows MODE 0): the launch dispatch per layer and
// input width. Kernel body: conv_rows.h.
#include "conv_rows.h"

DCUE_KTRACE_READER(fwd)  // diagnostic builds only (dcue_common.h)

namespace dcue {

template <int L, int KC, int SRC, int TW>
static int fwd_layer_tw(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  static_assert(KC % 32 == 0, "split-f16 chunks are 32 channels");
  if (a.wpack16 && conv_f16_on())
    return run_rows<0, SRC, KC, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, TW, 1, 1, true>(a, s);
  return run_rows<0, SRC, KC, gm.ks, gm.pad, gm.lin, gm.lp * gm.pool, gm.pool, TW, 1, 1>(a, s);
}

template <int L, int KC, int SRC>
static int fwd_layer(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int TWMAX = max_tw(gm.lp * gm.pool, gm.ks, KC);
  const int tw = choose_tw((long)a.M * gm.lp * gm.pool, TWMAX);
  if constexpr (TWMAX >= 8) if (tw == 8) return fwd_layer_tw<L, KC, SRC, 8>(a, s);
  if constexpr (TWMAX >= 4) if (tw == 4) return fwd_layer_tw<L, KC, SRC, 4>(a, s);
  if constexpr (TWMAX >= 3) if (tw == 3) return fwd_layer_tw<L, KC, SRC, 3>(a, s);
  if constexpr (TWMAX >= 2) if (tw == 2) return fwd_layer_tw<L, KC, SRC, 2>(a, s);
  return fwd_layer_tw<L, KC, SRC, 1>(a, s);
}

template <int L>
static int fwd_kc(int kc, int src, const RowsArgs& a, hipStream_t s) {
  if constexpr (L == 1) {
    if (kc != kMels) return DCUE_ERR_INVALID;
    return src == SRC_TRACK_F16 ? fwd_layer<1, 128, SRC_TRACK_F16>(a, s)
                                : fwd_layer<1, 128, SRC_TRACK_F32>(a, s);
  } else {
    switch (kc) {
      case 32: return fwd_layer<L, 32, SRC_ACT>(a, s);
      case 64: return fwd_layer<L, 64, SRC_ACT>(a, s);
      case 128: return fwd_layer<L, 128, SRC_ACT>(a, s);
      case 256: return fwd_layer<L, 256, SRC_ACT>(a, s);
      default: return DCUE_ERR_UNSUPPORTED;
    }
  }
}

int launch_conv_fwd(int layer, int kc, int src, const RowsArgs& a, hipStream_t s) {
  switch (layer) {
    case 1: return fwd_kc<1>(kc, src, a, s);
    case 2: return fwd_kc<2>(kc, src, a, s);
    case 3: return fwd_kc<3>(kc, src, a, s);
    case 4: return fwd_kc<4>(kc, src, a, s);
    case 5: return fwd_kc<5>(kc, src, a, s);
    default: return DCUE_ERR_INVALID;
  }
}

}  // namespace dcue

