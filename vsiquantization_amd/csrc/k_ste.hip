// k_ste.hip — straight-through backward from the saved 1-bit mask, and its C ABI.
#include "vsiq_common.cuh"

namespace vsiq {

// ----------------------------------------------------------------------------
// STE backward with the saved 1-bit mask: gx = (m ? g*s : 0) / s, grid (rows, chunks)
// (division: ste_quot in vsiq_common.cuh)
// ----------------------------------------------------------------------------
// one-shot: workgroup b covers chunk b % chunks of row b / chunks (U groups per lane:
// kFlatU, or 9 for a one-round grid with a store gate or deferred store phase, see
// store_gate / defer_stores).
// A wave's 64 groups are one 256-element mask chunk: its four mask words are
// wave-uniform, read with scalar loads and used directly as lane masks.
// ACT (K5): `pre` holds the pre-activation c of a fused ReLU/SiLU; the result is
// the activation's backward applied to the quantizer's grad_x.
template <bool VEC, bool NT, int ACT, int U>
__global__ __launch_bounds__(kBlock) void k_ste_bwd(const float *__restrict__ g,
                                                    const uint64_t *__restrict__ mask,
                                                    const float *__restrict__ pre,
                                                    float *__restrict__ gx, int64_t rowlen,
                                                    uint32_t chunks, const double *__restrict__ sdev,
                                                    double shost, uint32_t defer, uint32_t gate, SiluLay L) {
  const GateClk gc = gate_begin(gate);
  const int64_t row = blockIdx.x / chunks;
  const int64_t chunk = blockIdx.x % chunks;
  const SteDiv d = make_stediv((float)(sdev ? sdev[row] : shost));
  const int64_t ng = cdiv(rowlen, 4);
  const int64_t nchunk = cdiv(ng, kWave);
  const float *gr = g + row * rowlen;
  float *xr = gx + row * rowlen;
  const uint64_t *mr = mask + row * mask_words_per_row(rowlen);
  const int64_t base = chunk * kBlock * U + threadIdx.x;
  const int wave0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  f4 v[U], cv[U];
  uint64_t w[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kBlock;
    v[u] = load_group<VEC, NT>(gr, i < ng ? i : ng - 1, rowlen);
    if (ACT) cv[u] = load_group<VEC, NT>(pre + row * rowlen, i < ng ? i : ng - 1, rowlen);
    int64_t c = chunk * (kBlock / kWave) * U + u * (kBlock / kWave) + wave0;
    c = c < nchunk ? c : nchunk - 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[u][j] = mr[4 * c + j];
  }
  // all groups computed before the first store: a (predicated, hence branched-around)
  // store ahead of a load's use would make hipcc wait for the store as well
  f4 o[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool m0 = __builtin_amdgcn_inverse_ballot_w64(w[u][0]);
    const bool m1 = __builtin_amdgcn_inverse_ballot_w64(w[u][1]);
    const bool m2 = __builtin_amdgcn_inverse_ballot_w64(w[u][2]);
    const bool m3 = __builtin_amdgcn_inverse_ballot_w64(w[u][3]);
    o[u].x = m0 ? ste_quot(v[u].x, d) : 0.0f;
    o[u].y = m1 ? ste_quot(v[u].y, d) : 0.0f;
    o[u].z = m2 ? ste_quot(v[u].z, d) : 0.0f;
    o[u].w = m3 ? ste_quot(v[u].w, d) : 0.0f;
    if (!(d.fast & ste_ok(v[u].x) & ste_ok(v[u].y) & ste_ok(v[u].z) & ste_ok(v[u].w))) {
      o[u].x = ste_ieee(v[u].x, m0, d);   // rare
      o[u].y = ste_ieee(v[u].y, m1, d);
      o[u].z = ste_ieee(v[u].z, m2, d);
      o[u].w = ste_ieee(v[u].w, m3, d);
    }
    if (ACT) o[u] = act_bwd4_at<ACT>(o[u], cv[u], row * rowlen + 4 * (base + u * kBlock), L);
  }
  if (defer) {   // kernel-uniform
    __syncthreads();
    defer_stores(defer);
  }
  gate_pass(gate, gc);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kBlock;
    if (i < ng) store_group<VEC, NT>(xr, i, rowlen, o[u]);
  }
}


template <int ACT, bool VEC, bool NT>
void launch_ste_act(const float *g, const uint64_t *m, const float *pre, float *gx, int64_t rows,
                    int64_t rowlen, const double *sdev, double shost, const SiluLay &L, hipStream_t st) {
  const int64_t ng = cdiv(rowlen, 4);
  const int64_t chunks9 = cdiv(ng, (int64_t)kBlock * 9);
  const bool fits9 = chunks9 * kBlock * 9 - ng <= ng / 8;
  GateSel gs;
  // one-round grids: store gate (auto; C2 STE 13.3-13.6 -> 12.9-13.0 us in bench.py on
  // MI355X), else the deferred store phase where that was measured to pay
  if (fits9 && g_tune.store_gate != 0) {
    const void *kern = reinterpret_cast<const void *>(k_ste_bwd<VEC, NT, ACT, 9>);
    static const int occ = occupancy_blocks(kern, kBlock);
    const int64_t bytes = rows * rowlen * (int64_t)(ACT ? 8 : 4) + rows * mask_words_per_row(rowlen) * 8;
    gs = store_gate_select("ste_bwd", kern, rows * chunks9, occ, bytes, st);
  }
  // "no gate" (also as a tuning candidate) = the deferred store phase where it applies
  const uint32_t defer = fits9 && !gs.gate ? store_defer_units(rows * chunks9, true) : 0;
  if (defer || gs.gate) {
    hipLaunchKernelGGL((k_ste_bwd<VEC, NT, ACT, 9>), dim3((unsigned)(rows * chunks9)), dim3(kBlock), 0, st,
                       g, m, pre, gx, rowlen, (uint32_t)chunks9, sdev, shost, defer, gs.gate, L);
  } else {
    const int64_t chunks = oneshot_grid(ng);
    hipLaunchKernelGGL((k_ste_bwd<VEC, NT, ACT, kFlatU>), dim3((unsigned)(rows * chunks)), dim3(kBlock), 0,
                       st, g, m, pre, gx, rowlen, (uint32_t)chunks, sdev, shost, 0u, 0u, L);
  }
  store_gate_launched(gs, st);
}

template <int ACT>
void launch_ste(bool vec, bool nt, const float *g, const uint64_t *m, const float *pre, float *gx,
                int64_t rows, int64_t rowlen, const double *sdev, double shost, const SiluLay &L, hipStream_t st) {
  if (vec && nt) launch_ste_act<ACT, true, true>(g, m, pre, gx, rows, rowlen, sdev, shost, L, st);
  else if (vec) launch_ste_act<ACT, true, false>(g, m, pre, gx, rows, rowlen, sdev, shost, L, st);
  else if (nt) launch_ste_act<ACT, false, true>(g, m, pre, gx, rows, rowlen, sdev, shost, L, st);
  else launch_ste_act<ACT, false, false>(g, m, pre, gx, rows, rowlen, sdev, shost, L, st);
}

int ste_bwd(const float *g, const uint64_t *mask, const float *pre, float *gx, int64_t n, int act,
            const double *scale_dev, int64_t rowlen, double scale_host, void *stream) {
  if (n < 0 || !act_ok(act)) return VSIQ_E_ARG;
  if (n == 0) return 0;
  if (!g || !mask || !gx || (act != kActNone && !pre)) return VSIQ_E_ARG;
  if (!aligned8(mask)) return VSIQ_E_ALIGN;
  if (!scale_dev || rowlen <= 0) rowlen = n;
  if (n % rowlen != 0) return VSIQ_E_ARG;
  const int64_t rows = n / rowlen;
  if (rows * oneshot_grid(cdiv(rowlen, 4)) > 0x7fffffffLL) return VSIQ_E_ARG;
  const bool vec = (rowlen % 4 == 0) && aligned16(g) && aligned16(gx) && (!pre || aligned16(pre));
  const bool nt = g_tune.nontemporal != 0;
  VSIQ_ACT(act, launch_ste, vec, nt, g, mask, pre, gx, rows, rowlen, scale_dev, scale_host,
           act_lay(act, n), (hipStream_t)stream);
  return launch_rc();
}

}  // namespace vsiq

using namespace vsiq;

extern "C" {

int vsiq_ste_bwd_f32(const float *g, const uint64_t *mask, float *gx, int64_t n,
                     const double *scale_dev, int64_t rowlen, double scale_host, void *stream) {
  return ste_bwd(g, mask, nullptr, gx, n, kActNone, scale_dev, rowlen, scale_host, stream);
}

int vsiq_act_ste_bwd_f32(const float *g, const uint64_t *mask, const float *c, float *gc, int64_t n,
                         int act, const double *scale_dev, int64_t rowlen, double scale_host,
                         void *stream) {
  return ste_bwd(g, mask, c, gc, n, act, scale_dev, rowlen, scale_host, stream);
}

}  // extern "C"
