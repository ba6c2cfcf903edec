// geometry.h — fp64 vector helpers, SDF primitives and the flattened SDF program.
//
// Every function follows the reference's operation order (file:line cited) and the library
// is built with -ffp-contract=off, so values are bit-identical to the CPU restatement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smcrt.h"
#include "detmath.h"

namespace smcrt {

struct V3 {
  double x, y, z;
};
__host__ __device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__host__ __device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__host__ __device__ __forceinline__ V3 mul(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }   // vec*scal
__host__ __device__ __forceinline__ V3 smul(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }  // scal*vec
__host__ __device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ double len(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
__host__ __device__ __forceinline__ V3 vabs(V3 a) { return v3(fabs(a.x), fabs(a.y), fabs(a.z)); }
__host__ __device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }
__host__ __device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }
__host__ __device__ __forceinline__ double clampd(double v, double lo, double hi) { return dmin(dmax(v, lo), hi); }

// vec_dot_mat, vector_class.f90:292-304 (transform column-major)
__host__ __device__ __forceinline__ V3 dotmat(V3 a, const double* t) {
  return v3(t[0] * a.x + t[1] * a.y + t[2] * a.z + t[3], t[4] * a.x + t[5] * a.y + t[6] * a.z + t[7],
            t[8] * a.x + t[9] * a.y + t[10] * a.z + t[11]);
}

// CSG operators, sdfModifiers.f90:428-491
__host__ __device__ __forceinline__ double csg(int32_t op, double d1, double d2, double k) {
  switch (op) {
    case SMCRT_OP_UNION: return dmin(d1, d2);
    case SMCRT_OP_SMOOTH_UNION: {
      const double h = dmax(k - fabs(d1 - d2), 0.0) / k;
      return dmin(d1, d2) - h * h * h * k * (1.0 / 6.0);
    }
    case SMCRT_OP_SUBTRACTION: return dmax(-d1, d2);
    default: return dmax(d1, d2);
  }
}

// One primitive, sdfs.f90:494-735, at p = pos .dot. transform. `nd` is wave-uniform: its
// fields arrive by scalar loads and the switch never diverges.
//
// translate_only: the transform's 3x3 part is the identity (every builder's
// invert(translate(c)), setupGeometry.f90:64,289), so ((x*1 + y*0) + z*0) + t = x + t.
// This is exact for every finite input; at most the sign of a zero result differs, which
// no SDF below can observe (they use squares, abs, min/max and comparisons with 0).
//
// sdf_prim_s reads the primitive's kind, transform t[0..11] and parameters P[0..7] with a
// stride of S doubles (S = 1: a node; S = 64: the cooperative EVAL's LDS table, one column
// per lane, transport.h); sdf_prim is it applied to a node.
// sdf_shape_s is the primitive's formula at its local point p; sdf_prim_s forms p first.
template <int S>
__host__ __device__ __forceinline__ double sdf_shape_s(int32_t kind, const double* __restrict__ P_, const V3 p) {
#define P(i) P_[(i) * S]
  switch (kind) {
    case SMCRT_SDF_SPHERE:  // :494-508
      return sqrt(p.x * p.x + p.y * p.y + p.z * p.z) - P(0);
    case SMCRT_SDF_BOX: {  // :510-525
      const V3 q = vabs(p) - v3(P(0), P(1), P(2));
      const double mx = dmax(q.x, 0.0), my = dmax(q.y, 0.0), mz = dmax(q.z, 0.0);
      const double s2 = mx * mx + my * my + mz * mz;  // len(max(q, 0)) = sqrt(s2)
      double l = 0.0;
#ifdef __HIP_DEVICE_COMPILE__
      // a point inside the box has s2 = +0 and sqrt(+0) = +0: the (costly) fp64 square root
      // is skipped when no lane of the wave needs it, with the same bits
      if (__ballot(s2 != 0.0)) l = sqrt(s2);
#else
      l = sqrt(s2);
#endif
      return l + dmin(dmax(q.x, dmax(q.y, q.z)), 0.0);
    }
    case SMCRT_SDF_TORUS: {  // :527-542
      const V3 q = v3(len(v3(p.x, 0.0, p.z)) - P(0), p.y, 0.0);
      return len(q) - P(1);
    }
    case SMCRT_SDF_CYLINDER: {  // :544-581
      const V3 a = v3(P(0), P(1), P(2)), b = v3(P(3), P(4), P(5));
      const V3 ba = b - a, pa = p - a;
      const double baba = dot(ba, ba), paba = dot(pa, ba);
      const double x = len(mul(pa, baba) - mul(ba, paba)) - P(6) * baba;
      const double y = fabs(paba - baba * 0.5) - baba * 0.5;
      const double x2 = x * x, y2 = (y * y) * baba;
      double d;
      if (dmax(x, y) < 0.0) d = -dmin(x2, y2);
      else if (x > 0.0 && y > 0.0) d = x2 + y2;
      else if (x > 0.0) d = x2;
      else if (y > 0.0) d = y2;
      else d = 0.0;
      return copysign(sqrt(fabs(d)) / baba, d);
    }
    case SMCRT_SDF_TRIPRISM: {  // :583-597
      const V3 q = vabs(p);
      return dmax(q.z - P(1), dmax(q.x * 0.866025 + p.y * 0.5, -p.y) - P(0) * 0.5);
    }
    case SMCRT_SDF_SEGMENT: {  // :599-626
      const V3 a = v3(P(0), P(1), P(2)), b = v3(P(3), P(4), P(5));
      const V3 pa = p - a, ba = b - a;
      const double h = clampd(dot(pa, ba) / dot(ba, ba), 0.0, 1.0);
      return len(pa - mul(ba, h)) - 0.1;
    }
    case SMCRT_SDF_CAPSULE: {  // :628-648
      const V3 a = v3(P(0), P(1), P(2)), b = v3(P(3), P(4), P(5));
      const V3 pa = p - a, ba = b - a;
      const double h = clampd(dot(pa, ba) / dot(ba, ba), 0.0, 1.0);
      return len(pa - mul(ba, h)) - P(6);
    }
    case SMCRT_SDF_CONE: {  // :650-686
      const V3 a = v3(P(0), P(1), P(2)), b = v3(P(3), P(4), P(5));
      const double ra = P(6), rb = P(7);
      const double rba = rb - ra;
      const double baba = dot(b - a, b - a);
      const double papa = dot(p - a, p - a);
      const double paba = dot(p - a, b - a) / baba;
      const double x = sqrt(papa - baba * (paba * paba));
      const double cax = (paba < 0.5) ? dmax(0.0, x - ra) : dmax(0.0, x - rb);
      const double cay = fabs(paba - 0.5) - 0.5;
      const double k = rba * rba + baba;
      const double f = clampd((rba * (x - ra) + paba * baba) / k, 0.0, 1.0);
      const double cbx = x - ra - f * rba;
      const double cby = paba - f;
      const double s = (cbx < 0.0 && cay < 0.0) ? -1.0 : 1.0;
      return s * sqrt(dmin(cax * cax + baba * (cay * cay), cbx * cbx + baba * (cby * cby)));
    }
    case SMCRT_SDF_EGG: {  // :688-718
      const double r1 = P(0), r2 = P(1), hh = P(2);
      const V3 pin = v3(fabs(p.x), p.y, p.z);
      const double r = r1 - r2;
      const double h_in = hh + r;
      const double l = (h_in * h_in - r * r) / (2.0 * r);
      if (pin.y <= 0.0) return len(pin) - r1;
      if ((pin.y - h_in) * l > pin.x * h_in) return len(pin - v3(0.0, h_in, 0.0)) - ((r1 + l) - len(v3(h_in, l, 0.0)));
      return len(pin + v3(l, 0.0, 0.0)) - (r1 + l);
    }
    case SMCRT_SDF_PLANE:  // :720-735
      return dot(p, v3(P(0), P(1), P(2)));
    default:
      return __builtin_nan("");
  }
#undef P
}

template <int S>
__host__ __device__ __forceinline__ double sdf_prim_s(int32_t kind, const double* __restrict__ t,
                                                      const double* __restrict__ P_, V3 pos, bool translate_only) {
#define T(i) t[(i) * S]
  const V3 p = translate_only ? v3(pos.x + T(3), pos.y + T(7), pos.z + T(11))
                              : v3(T(0) * pos.x + T(1) * pos.y + T(2) * pos.z + T(3),
                                   T(4) * pos.x + T(5) * pos.y + T(6) * pos.z + T(7),
                                   T(8) * pos.x + T(9) * pos.y + T(10) * pos.z + T(11));  // dotmat
#undef T
  return sdf_shape_s<S>(kind, P_, p);
}

__host__ __device__ __forceinline__ double sdf_prim(const smcrt_sdf_node* __restrict__ nd, V3 pos, bool translate_only) {
  return sdf_prim_s<1>(nd->kind, nd->transform, nd->param, pos, translate_only);
}


// The SDF array flattened into one instruction stream, so the kernel evaluates every
// top-level SDF (and every CSG child, folded left to right as eval_model does,
// sdf_base.f90:146-161) with a single inlined copy of sdf_prim.
enum : int32_t {
  PROG_TOP = 0,         // primitive that is itself a top-level SDF
  PROG_CHILD_FIRST = 1, // first child of a model: acc = d
  PROG_CHILD = 2,       // later child: acc = op(acc, d)
};
// Nested composites (a model among a model's children: eval_model recurses through
// array(i)%value%evaluate, sdf_base.f90:146-161; or a modifier of sdfModifiers.f90, which
// wraps one node). A top-level model's children are ops of the program; a child that is
// itself a composite, or a top-level modifier, is one op with PROG_SUB whose value node_value
// computes. Composites may nest PROG_MAX_DEPTH levels below a top (the reference's recursion
// has no limit; scene creation rejects deeper trees and trees that contain themselves).
enum : int32_t { PROG_SUB = 8 };
constexpr int PROG_MAX_DEPTH = 32;

struct ProgOp {
  int32_t node;   // primitive node index
  int32_t action; // PROG_* (| PROG_NEST ...)
  int32_t top;    // 1-based top-level index completed by this op (0 if none)
  int32_t op;     // CSG op for PROG_CHILD
  double k;       // CSG parameter
  int32_t translate_only;  // the node's transform is a pure translation (see sdf_prim)
  int32_t pad;
};

// Models and modifiers ("composite" nodes, every kind from SMCRT_SDF_MODEL on).
__host__ __device__ __forceinline__ bool composite_kind(int32_t kind) { return kind >= SMCRT_SDF_MODEL; }

// A modifier's query point for its wrapped node (sdfModifiers.f90). Revolution :303-321,
// elongate :335-351 (max(q, 0)), twist :353-371, bend :373-391; the others pass pos through.
__host__ __device__ __forceinline__ V3 modifier_point(const smcrt_sdf_node* __restrict__ M, V3 pos) {
  const double* P = M->param;
  switch (M->kind) {
    case SMCRT_SDF_REVOLUTION: {  // p_in = pos - center; q = (length(p_in.xz) - o, p_in.y, 0)
      const V3 pin = pos - v3(P[1], P[2], P[3]);
      return v3(len(v3(pin.x, 0.0, pin.z)) - P[0], pin.y, 0.0);
    }
    case SMCRT_SDF_ELONGATE: {  // q = abs(pos) - size; the wrapped node sees max(q, 0)
      const V3 q = vabs(pos) - v3(P[0], P[1], P[2]);
      return v3(dmax(q.x, 0.0), dmax(q.y, 0.0), dmax(q.z, 0.0));
    }
    case SMCRT_SDF_TWIST:
    case SMCRT_SDF_BEND: {  // c = cos(k*a), s = sin(k*a), a = pos%z (twist) or pos%x (bend)
      double sn, cs;
      det_sincos_any(P[0] * (M->kind == SMCRT_SDF_TWIST ? pos.z : pos.x), &sn, &cs);
      return v3(cs * pos.x - sn * pos.y, sn * pos.x + cs * pos.y, pos.z);
    }
    default:
      return pos;
  }
}

// A modifier's value from its wrapped node's value d at its own query point pos.
// Extrude :286-301, onion :323-333, elongate :335-351 (+ w), displacement :393-408.
__host__ __device__ __forceinline__ double modifier_value(const smcrt_sdf_node* __restrict__ M, double d, V3 pos) {
  const double* P = M->param;
  switch (M->kind) {
    case SMCRT_SDF_EXTRUDE: {  // w = (d, abs(pos%z) - h, 0); min(max(w%x, w%y), 0) + length(max(w, 0))
      const double wy = fabs(pos.z) - P[0];
      return dmin(dmax(d, wy), 0.0) + len(v3(dmax(d, 0.0), dmax(wy, 0.0), dmax(0.0, 0.0)));
    }
    case SMCRT_SDF_ONION:  // abs(d) - thickness
      return fabs(d) - P[0];
    case SMCRT_SDF_ELONGATE: {  // + min(max(q%x, max(q%y, q%z)), 0)
      const V3 q = vabs(pos) - v3(P[0], P[1], P[2]);
      return d + dmin(dmax(q.x, dmax(q.y, q.z)), 0.0);
    }
    case SMCRT_SDF_DISPLACEMENT: {  // d1 + d2, d2 = the built-in f(pos) (smcrt.h smcrt_displacement_fn)
      double sx, sy, sz, c;
      det_sincos_any(P[2] * pos.x, &sx, &c);
      det_sincos_any(P[3] * pos.y, &sy, &c);
      det_sincos_any(P[4] * pos.z, &sz, &c);
      return d + ((P[1] * sx) * sy) * sz;
    }
    default:  // revolution, twist, bend: the wrapped node's value
      return d;
  }
}

// The value of node `idx` at pos: a primitive (its own transform), a model (eval_model's left
// fold over its children, sdf_base.f90:146-161; the model's transform is not applied) or a
// modifier (its wrapped node at modifier_point, then modifier_value). Composites are walked
// without recursion: a stack of frames (node, next child, accumulator, query point), one per
// open composite, so the depth costs stack slots (private memory), not inlined code, and
// every level runs the same single primitive site. The operations and their order are those
// of the recursive definition, so the value is the same bit for bit. Children are evaluated
// with their transforms in full (dotmat), which equals sdf_prim's translate-only shortcut bit
// for bit (see sdf_prim_s). A tree deeper than PROG_MAX_DEPTH (rejected at scene creation)
// yields NaN.
struct NodeFrame {
  int32_t idx, c;  // the composite, its next child
  double acc;      // the fold of its children so far
  V3 pos;          // the point it is evaluated at
};
__host__ __device__ __forceinline__ double node_value(const smcrt_sdf_node* __restrict__ nodes, int32_t idx, V3 pos) {
  if (!composite_kind(nodes[idx].kind)) return sdf_prim(nodes + idx, pos, false);
  NodeFrame st[PROG_MAX_DEPTH];
  int sp = 0;
  st[0].idx = idx; st[0].c = 0; st[0].acc = 0.0; st[0].pos = pos;
  for (;;) {
    const smcrt_sdf_node* __restrict__ M = nodes + st[sp].idx;
    const bool model = M->kind == SMCRT_SDF_MODEL;
    double v;
    if (st[sp].c < (model ? M->n_children : 1)) {
      const int32_t ci = M->first_child + st[sp].c;
      const V3 q = model ? st[sp].pos : modifier_point(M, st[sp].pos);
      if (composite_kind(nodes[ci].kind)) {  // open the child composite
        if (sp + 1 >= PROG_MAX_DEPTH) return __builtin_nan("");
        ++sp;
        st[sp].idx = ci; st[sp].c = 0; st[sp].acc = 0.0; st[sp].pos = q;
        continue;
      }
      v = sdf_prim(nodes + ci, q, false);  // a primitive child: folded into this frame
    } else {  // every child folded: the composite's value goes to its parent frame
      v = model ? st[sp].acc : modifier_value(M, st[sp].acc, st[sp].pos);
      if (sp == 0) return v;
      --sp;
    }
    const smcrt_sdf_node* __restrict__ P = nodes + st[sp].idx;
    st[sp].acc = (st[sp].c == 0 || P->kind != SMCRT_SDF_MODEL) ? v : csg(P->op, st[sp].acc, v, P->k);
    ++st[sp].c;
  }
}

// The value an op contributes: its primitive, or (PROG_SUB) its composite node's value: a
// model among a top model's children, or a top-level modifier (node_value).
// NEST = false (every kernel but the general instantiation, which scenes with composites below
// the top level always use, smcrt.hip) compiles only the primitive.
template <bool NEST>
__host__ __device__ __forceinline__ double prog_value(const smcrt_sdf_node* __restrict__ nodes, int32_t node,
                                                      int32_t action, bool translate_only, V3 q) {
  if constexpr (!NEST) return sdf_prim(nodes + node, q, translate_only);
  if (!(action & PROG_SUB)) return sdf_prim(nodes + node, q, translate_only);
  return node_value(nodes, node, q);
}

}  // namespace smcrt
