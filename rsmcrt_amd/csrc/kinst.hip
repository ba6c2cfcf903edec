// kinst.hip — one (LDS faces, grid mode) slice of the transport kernel instantiations.
// Compiled twelve times by build.py (-DKI_F=0/1 -DKI_G=0/1/2 -DKI_P=0/1); see kernel_ptrs.h.
// Part 0 holds transport_kernel and the XF ws_kernel, part 1 the plain ws_kernel (the lean path
// of M1), which build.py compiles with its own scheduler flags (see UNITS there).
#include "kernels.h"
#include "kernel_ptrs.h"

#if !defined(KI_F) || !defined(KI_G) || !defined(KI_P)
#error "kinst.hip is compiled with -DKI_F=<0|1> -DKI_G=<0|1|2> -DKI_P=<0|1> (rsmcrt_amd/build.py)"
#endif
#define KI_NAME3(a, f, g) a##_##f##_##g
#define KI_NAME2(a, f, g) KI_NAME3(a, f, g)
#define KI_NAME(a) KI_NAME2(a, KI_F, KI_G)

namespace smcrt {

#if KI_P == 1
// the plain ws_kernel (no Fresnel program points, no detectors)
const void* KI_NAME(kinst_wsp)(int slots) {
  return slots == 3 ? (const void*)ws_kernel<KI_F != 0, KI_G, false, 3> : (const void*)ws_kernel<KI_F != 0, KI_G, false, 2>;
}
#define KI_DIAG_NAME KI_NAME(kinst_diagp)
#else
const void* KI_NAME(kinst_transport)(int xsrc, int coop) {
  constexpr bool F = KI_F != 0;
  if (xsrc && coop) {
    if constexpr (!F) return (const void*)transport_kernel<false, KI_G, true, true>;
    return nullptr;
  }
  if (xsrc) return (const void*)transport_kernel<F, KI_G, true, false>;
  if (coop) return (const void*)transport_kernel<F, KI_G, false, true>;
  return (const void*)transport_kernel<F, KI_G, false, false>;
}

#if KI_F == 0 && KI_G == 0
size_t kinst_ws_shared_bytes(int slots) { return slots == 3 ? sizeof(WsSharedT<3>) : sizeof(WsSharedT<2>); }
int kinst_ws_threads() { return WS_THREADS; }
int kinst_ws_photon_lanes() { return (int)WS_NPL; }
size_t kinst_ws_scratch_bytes(size_t lanes) { return ws_scratch_bytes(lanes); }
#endif

const void* KI_NAME(kinst_ws)(int xf, int slots) {
  if (xf) return slots == 3 ? (const void*)ws_kernel<KI_F != 0, KI_G, true, 3> : (const void*)ws_kernel<KI_F != 0, KI_G, true, 2>;
  return KI_NAME(kinst_wsp)(slots);
}
#define KI_DIAG_NAME KI_NAME(kinst_diag)
#endif


// (each part has its own copy of the static tallies)
void KI_DIAG_NAME(unsigned long long* d72, unsigned long long* t9, unsigned long long* c6) {
#ifdef SMCRT_DIAG
  unsigned long long h[72] = {0}, z[72] = {0};
  if (hipDeviceSynchronize() != hipSuccess) return;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag), sizeof(h)) == hipSuccess)
    for (int i = 0; i < 72; ++i) d72[i] += (i >= 68 && i <= 69) ? 0 : h[i];
  for (int i = 68; i <= 69; ++i) d72[i] = h[i] > d72[i] ? h[i] : d72[i];  // the longest wave: a max
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof(z));
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag_t), sizeof(unsigned long long) * 9) == hipSuccess)
    for (int i = 0; i < 9; ++i) t9[i] += h[i];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag_t), z, sizeof(unsigned long long) * 9);
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cull_diag), sizeof(unsigned long long) * 6) == hipSuccess)
    for (int i = 0; i < 6; ++i) c6[i] += h[i];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cull_diag), z, sizeof(unsigned long long) * 6);
#else
  (void)d72; (void)t9; (void)c6;
#endif
}

}  // namespace smcrt
