// Forward convolutions of the item tower (k_conv_rows MODE 0): the launch dispatch per layer and
// input width. Kernel body: conv_rows.h.
#include <algorithm>

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

#include "tgemm.h"

namespace dcue {

// ------------------------------------------------------------- in-batch forward tail, fused
// Conv 4 (+ BN3 applied, BN4 sums), conv 5 (+ BN4 applied, BN5 sums) and the fc on BN5(y5) in ONE
// workgroup: at in-batch M <= 64 conv 4's 2M rows fit one workgroup's eight 16-row tiles and conv
// 5's M rows four, so each layer's BatchNorm statistics are complete inside the workgroup -- no grid
// barrier, and two kernel boundaries fewer on the forward chain (each a dispatch plus the first
// loads of a fresh kernel). The layers run conv_rows_body / tgemm_block,
// the device functions of the three launches it replaces, with the same tile maps: bit-identical
// results (DCUE_FWD_TAIL=0 runs the three launches). The fc's eight 16 x 64 blocks run two at a
// time (threads 0-255 / 256-511) over the slab's LDS.
template <int KC, bool F16>
__global__ __launch_bounds__(kRowsThreads) void k_fwd_tail(RowsArgs a4, RowsArgs a5, TGemmArgs fc) {
  extern __shared__ __attribute__((aligned(16))) float slab[];
  constexpr LayerGeom g4 = layer_geom(4), g5 = layer_geom(5);
  conv_rows_body<0, SRC_ACT, KC, g4.ks, g4.pad, g4.lin, g4.lp * g4.pool, g4.pool, 8, 1, 1, true, F16, true>(a4, 0, 0);
  __syncthreads();  // y4, its BN sums and range complete (this workgroup's own stores and atomics)
  conv_rows_body<0, SRC_ACT, KC, g5.ks, g5.pad, g5.lin, g5.lp * g5.pool, g5.pool, 4, 1, 1, true, F16, true>(a5, 0, 0);
  __syncthreads();
  TgLds* L = reinterpret_cast<TgLds*>(slab);
  const int half = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int bxn = (fc.M + 15) / 16, byn = (fc.N + 63) / 64;
  for (int b0 = 0; b0 < bxn * byn; b0 += 2) {  // (uniform: both halves run every pass's barriers)
    const int b = min(b0 + half, bxn * byn - 1);
    if (b0 + half < bxn * byn) {
      tgemm_block<2, 0, 1, 0>(fc, b % bxn, b / bxn, L[half], t);
    } else {  // an odd last block: the idle half still takes the block's barriers (two per K stage)
      for (int k0 = 0; k0 < fc.K; k0 += kTgKC) {
        __syncthreads();
        __syncthreads();
      }
    }
  }
}

bool fwd_tail_fits(int M, int H, int D, int nout4) {
  static const bool on = [] {
    const char* e = getenv("DCUE_FWD_TAIL");
    return !(e && e[0] == '0');
  }();
  return on && M >= 1 && M <= 64 && (H == 32 || H == 64 || H == 128) && nout4 == H && D <= 128 && D >= 1;
}

int launch_fwd_tail(const RowsArgs& a4, const RowsArgs& a5, const TGemmArgs& fc, int H, hipStream_t s) {
  if (fc.sak != 1 || fc.sbn == 1) return DCUE_ERR_INVALID;  // tgemm_block<2, 0, 1, 0>'s operand layouts
  const bool f16 = a4.wpack16 && a5.wpack16 && conv_f16_on();
  const size_t lds = std::max(slab_bytes(2, 2, H, 8), 2 * sizeof(TgLds));
  auto launch = [&](auto kern) -> int {
    static bool attr = false;
    if (!attr) {
      DCUE_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)std::max(slab_bytes(2, 2, 128, 8), 2 * sizeof(TgLds))));
      attr = true;
    }
    DCUE_LAUNCH(kern, dim3(1), dim3(kRowsThreads), lds, s, a4, a5, fc);
    DCUE_LAUNCH_CHECK();
    return DCUE_OK;
  };
  switch (H * 2 + (f16 ? 1 : 0)) {
    case 64: return launch(k_fwd_tail<32, false>);
    case 65: return launch(k_fwd_tail<32, true>);
    case 128: return launch(k_fwd_tail<64, false>);
    case 129: return launch(k_fwd_tail<64, true>);
    case 256: return launch(k_fwd_tail<128, false>);
    case 257: return launch(k_fwd_tail<128, true>);
    default: return DCUE_ERR_UNSUPPORTED;
  }
}

}  // namespace dcue
