// kernel_ptrs.h — the transport kernel instantiations, reached through pointers.
//
// build.py compiles kinst.hip once per (LDS faces F, grid mode G, part P) with -DKI_F=F -DKI_G=G
// -DKI_P=P (part 1: the plain ws_kernel, with its own scheduler flags), so
// the instantiations of transport_kernel and ws_kernel (kernels.h, ws.h) build in parallel
// instead of in one translation unit. Each object exports these getters; hipLaunchKernel and
// the occupancy queries take the host stubs they return.
#pragma once
#include <stddef.h>

namespace smcrt {

size_t kinst_ws_shared_bytes(int slots);  // sizeof(WsSharedT<slots>), ws_kernel's static LDS (slots 2 or 3)
int kinst_ws_threads();            // ws_kernel's block size
int kinst_ws_photon_lanes();       // photon lanes per ws_kernel block
size_t kinst_ws_scratch_bytes(size_t lanes);  // ws_kernel lane scratch (ws.h WX_*) of that many photon lanes

#define SMCRT_KINST_DECL(F, G)                                                               \
  const void* kinst_transport_##F##_##G(int xsrc, int coop);                                 \
  const void* kinst_ws_##F##_##G(int xf, int slots);                                         \
  const void* kinst_wsp_##F##_##G(int slots);                                                \
  void kinst_diag_##F##_##G(unsigned long long* d72, unsigned long long* t9, unsigned long long* c6); \
  void kinst_diagp_##F##_##G(unsigned long long* d72, unsigned long long* t9, unsigned long long* c6);
SMCRT_KINST_DECL(0, 0)
SMCRT_KINST_DECL(0, 1)
SMCRT_KINST_DECL(0, 2)
SMCRT_KINST_DECL(1, 0)
SMCRT_KINST_DECL(1, 1)
SMCRT_KINST_DECL(1, 2)
#undef SMCRT_KINST_DECL

// transport_kernel<lds_faces, gm, xsrc, coop>; the general emitter with the COOP machinery
// (xsrc && coop) exists with faces in device memory only
inline const void* transport_kernel_ptr(bool lds_faces, int gm, bool xsrc, bool coop) {
  if (xsrc && coop) lds_faces = false;
  const int x = xsrc ? 1 : 0, c = coop ? 1 : 0;
  switch ((lds_faces ? 3 : 0) + gm) {
    case 0: return kinst_transport_0_0(x, c);
    case 1: return kinst_transport_0_1(x, c);
    case 2: return kinst_transport_0_2(x, c);
    case 3: return kinst_transport_1_0(x, c);
    case 4: return kinst_transport_1_1(x, c);
    default: return kinst_transport_1_2(x, c);
  }
}
// ws_kernel<lds_faces, gm, xf, slots> (xf: the Fresnel/detector program points; slots 2 or 3, ws.h)
inline const void* ws_kernel_ptr(bool lds_faces, int gm, bool xf, int slots) {
  const int x = xf ? 1 : 0;
  switch ((lds_faces ? 3 : 0) + gm) {
    case 0: return kinst_ws_0_0(x, slots);
    case 1: return kinst_ws_0_1(x, slots);
    case 2: return kinst_ws_0_2(x, slots);
    case 3: return kinst_ws_1_0(x, slots);
    case 4: return kinst_ws_1_1(x, slots);
    default: return kinst_ws_1_2(x, slots);
  }
}
// diagnostic builds: the kernels' tallies summed over the objects (each is cleared)
inline void kinst_diag_gather(unsigned long long* d72, unsigned long long* t9, unsigned long long* c6) {
  for (int i = 0; i < 72; ++i) d72[i] = 0;
  for (int i = 0; i < 9; ++i) t9[i] = 0;
  for (int i = 0; i < 6; ++i) c6[i] = 0;
  kinst_diag_0_0(d72, t9, c6); kinst_diag_0_1(d72, t9, c6); kinst_diag_0_2(d72, t9, c6);
  kinst_diag_1_0(d72, t9, c6); kinst_diag_1_1(d72, t9, c6); kinst_diag_1_2(d72, t9, c6);
  kinst_diagp_0_0(d72, t9, c6); kinst_diagp_0_1(d72, t9, c6); kinst_diagp_0_2(d72, t9, c6);
  kinst_diagp_1_0(d72, t9, c6); kinst_diagp_1_1(d72, t9, c6); kinst_diagp_1_2(d72, t9, c6);
}

}  // namespace smcrt
