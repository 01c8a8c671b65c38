// Input gradients of conv layers 2..5 (k_conv_rows MODE 1): the launch dispatch. Kernel body:
// conv_rows.h.
#include "conv_rows.h"

DCUE_KTRACE_READER(dgrad)  // diagnostic builds only (dcue_common.h)

namespace dcue {

// dgrad of layer L: rows = (item, input position t' < Lin_L), slab = layer-L conv positions
// [0, Lp*pool) carrying dz, taps reversed (PADL = ks-1-pad).
// Split-f16 MFMA (conv_rows.h F16: three f16 products per 32-channel chunk, the dz slab scaled by a
// power of two from the dz bound, range_stage) unless DCUE_DGRAD_F16=0 selects the exact-f32 path
static bool dgrad_f16_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_DGRAD_F16");
    return !(e && e[0] == '0');
  }();
  return on;
}

constexpr long kDgradF16MinRows = 8192;  // output rows M * Lin of a launch

template <int L, int KC, int TW>
static int dgrad_layer_tw(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  static_assert(KC % 32 == 0, "split-f16 chunks are 32 channels");
  // (small launches stay on f32: in-batch, the split's range stage and fill cost the one-tile
  // workgroups 1-3 us each, rocprof; catalogue layer 2: 128 -> 54 us)
  if (a.wpack16 && a.in_range && dgrad_f16_on() && (long)a.M * gm.lin >= kDgradF16MinRows)
    return run_rows<1, SRC_DZ, KC, gm.ks, gm.ks - 1 - gm.pad, gm.lp * gm.pool, gm.lin, 1, TW, gm.lp,
                    gm.pool, true>(a, s);
  return run_rows<1, SRC_DZ, KC, gm.ks, gm.ks - 1 - gm.pad, gm.lp * gm.pool, gm.lin, 1, TW, gm.lp,
                  gm.pool>(a, s);
}

template <int L, int KC>
static int dgrad_layer(const RowsArgs& a, hipStream_t s) {
  constexpr LayerGeom gm = layer_geom(L);
  constexpr int TWMAX = max_tw(gm.lin, gm.ks, KC);
  const int tw = choose_tw((long)a.M * gm.lin, TWMAX);
  if constexpr (TWMAX >= 8) if (tw == 8) return dgrad_layer_tw<L, KC, 8>(a, s);
  if constexpr (TWMAX >= 4) if (tw == 4) return dgrad_layer_tw<L, KC, 4>(a, s);
  if constexpr (TWMAX >= 3) if (tw == 3) return dgrad_layer_tw<L, KC, 3>(a, s);
  if constexpr (TWMAX >= 2) if (tw == 2) return dgrad_layer_tw<L, KC, 2>(a, s);
  return dgrad_layer_tw<L, KC, 1>(a, s);
}

template <int L>
static int dgrad_kc(int kc, const RowsArgs& a, hipStream_t s) {
  switch (kc) {
    case 32: return dgrad_layer<L, 32>(a, s);
    case 64: return dgrad_layer<L, 64>(a, s);
    case 128: return dgrad_layer<L, 128>(a, s);
    case 256: return dgrad_layer<L, 256>(a, s);
    default: return DCUE_ERR_UNSUPPORTED;
  }
}

int launch_conv_dgrad(int layer, int kc, const RowsArgs& a, hipStream_t s) {
  switch (layer) {
    case 2: return dgrad_kc<2>(kc, a, s);
    case 3: return dgrad_kc<3>(kc, a, s);
    case 4: return dgrad_kc<4>(kc, a, s);
    case 5: return dgrad_kc<5>(kc, a, s);
    default: return DCUE_ERR_INVALID;
  }
}

}  // namespace dcue

