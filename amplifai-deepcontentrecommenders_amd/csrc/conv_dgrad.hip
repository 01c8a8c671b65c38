// Input gradients of conv layers 2..5 (k_conv_rows MODE 1): the launch dispatch. Kernel body:
// conv_rows.h.
#include <algorithm>

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

namespace dcue {

// ------------------------------------------------------------- in-batch input-gradient tail, fused
// The input gradients of conv 5 (g4 + BN4's backward sums) and conv 4 (g3 + BN3's) in ONE workgroup:
// at in-batch M <= 64 their M and 2M output rows fit four and eight 16-row tiles, and conv 4's
// BN-backward operand (BN4's sums) is complete inside the workgroup once conv 5's part is done -- one
// kernel boundary fewer on the backward chain. conv_rows_body with the separate launches' tile maps
// (the f32 path they take at these sizes): bit-identical (DCUE_DGRAD_TAIL=0 runs the two launches).
template <int KC5, int KC4>
__global__ __launch_bounds__(kRowsThreads) void k_dgrad_tail(RowsArgs a5, RowsArgs a4) {
  constexpr LayerGeom g5 = layer_geom(5), g4 = layer_geom(4);
  conv_rows_body<1, SRC_DZ, KC5, g5.ks, g5.ks - 1 - g5.pad, g5.lp * g5.pool, g5.lin, 1, 4, g5.lp, g5.pool, true,
                 false, true>(a5, 0, 0);
  __syncthreads();  // g4, BN4's backward sums and max |g4| complete (this workgroup's own writes)
  conv_rows_body<1, SRC_DZ, KC4, g4.ks, g4.ks - 1 - g4.pad, g4.lp * g4.pool, g4.lin, 1, 8, g4.lp, g4.pool, true,
                 false, true>(a4, 0, 0);
}

bool dgrad_tail_fits(int M, int H, int D) {
  static const bool on = [] {
    const char* e = getenv("DCUE_DGRAD_TAIL");
    return !(e && e[0] == '0');
  }();
  return on && M >= 1 && M <= 64 && (H == 32 || H == 64 || H == 128) && (D == 32 || D == 64 || D == 128) &&
         (long)M * layer_geom(4).lin < kDgradF16MinRows;
}

int launch_dgrad_tail(const RowsArgs& a5, const RowsArgs& a4, int H, int D, hipStream_t s) {
  const size_t lds = std::max(slab_bytes(layer_geom(5).lin, layer_geom(5).ks, D, 4),
                              slab_bytes(layer_geom(4).lin, layer_geom(4).ks, H, 8));
  auto launch = [&](auto kern) -> int {
    static bool attr = false;
    if (!attr) {
      DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)std::max(slab_bytes(1, 1, 128, 4), slab_bytes(2, 2, 128, 8))));
      attr = true;
    }
    DCUE_LAUNCH(kern, dim3(1), dim3(kRowsThreads), lds, s, a5, a4);
    DCUE_LAUNCH_CHECK();
    return DCUE_OK;
  };
  switch (D * 1000 + H) {
    case 32032: return launch(k_dgrad_tail<32, 32>);
    case 32064: return launch(k_dgrad_tail<32, 64>);
    case 32128: return launch(k_dgrad_tail<32, 128>);
    case 64032: return launch(k_dgrad_tail<64, 32>);
    case 64064: return launch(k_dgrad_tail<64, 64>);
    case 64128: return launch(k_dgrad_tail<64, 128>);
    case 128032: return launch(k_dgrad_tail<128, 32>);
    case 128064: return launch(k_dgrad_tail<128, 64>);
    case 128128: return launch(k_dgrad_tail<128, 128>);
    default: return DCUE_ERR_UNSUPPORTED;
  }
}

}  // namespace dcue
