// mat4.h — host-side 4x4 transforms of the reference (vector_class.f90, mat_class.f90,
// sdfHelpers.f90), written term for term in the reference's operation order so that the
// matrices the SDF builders and the source emitters use are the reference's bits.
// Compiled with -ffp-contract=off like everything else.
#pragma once
#include <cmath>

namespace smcrt {
namespace mat {

// m[r][c] = Fortran t(r+1, c+1); stored column-major in smcrt_sdf_node.transform.
struct M4 {
  double m[4][4];
};

inline M4 identity() {
  M4 a{};
  for (int i = 0; i < 4; ++i) a.m[i][i] = 1.0;
  return a;
}

inline M4 translate(double x, double y, double z) {  // sdfHelpers.f90:160-171: row 4 holds o
  M4 a = identity();
  a.m[3][0] = x; a.m[3][1] = y; a.m[3][2] = z;
  return a;
}

inline M4 rotate_y(double angle) {  // sdfHelpers.f90:33-50, deg2rad(a) = a*pi/180
  const double r = angle * M_PI / 180.0, c = std::cos(r), s = std::sin(r);
  M4 a{};
  // columns (c,0,s,0) (0,1,0,0) (-s,0,c,0) (0,0,0,1)
  a.m[0][0] = c;  a.m[1][0] = 0; a.m[2][0] = s;  a.m[3][0] = 0;
  a.m[0][1] = 0;  a.m[1][1] = 1; a.m[2][1] = 0;  a.m[3][1] = 0;
  a.m[0][2] = -s; a.m[1][2] = 0; a.m[2][2] = c;  a.m[3][2] = 0;
  a.m[0][3] = 0;  a.m[1][3] = 0; a.m[2][3] = 0;  a.m[3][3] = 1;
  return a;
}

// Direct 4x4 inverse, term for term as mat_class.f90:154-207.
inline M4 invert(const M4& A) {
  auto a = [&](int i, int j) { return A.m[i - 1][j - 1]; };
  const double detinv =
      1.0 / (a(1, 1) * (a(2, 2) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3)) + a(2, 3) * (a(3, 4) * a(4, 2) - a(3, 2) * a(4, 4)) +
                        a(2, 4) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2))) -
             a(1, 2) * (a(2, 1) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3)) + a(2, 3) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4)) +
                        a(2, 4) * (a(3, 1) * a(4, 3) - a(3, 3) * a(4, 1))) +
             a(1, 3) * (a(2, 1) * (a(3, 2) * a(4, 4) - a(3, 4) * a(4, 2)) + a(2, 2) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4)) +
                        a(2, 4) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1))) -
             a(1, 4) * (a(2, 1) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2)) + a(2, 2) * (a(3, 3) * a(4, 1) - a(3, 1) * a(4, 3)) +
                        a(2, 3) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1))));
  M4 B{};
  B.m[0][0] = detinv * (a(2, 2) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3)) + a(2, 3) * (a(3, 4) * a(4, 2) - a(3, 2) * a(4, 4)) + a(2, 4) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2)));
  B.m[1][0] = detinv * (a(2, 1) * (a(3, 4) * a(4, 3) - a(3, 3) * a(4, 4)) + a(2, 3) * (a(3, 1) * a(4, 4) - a(3, 4) * a(4, 1)) + a(2, 4) * (a(3, 3) * a(4, 1) - a(3, 1) * a(4, 3)));
  B.m[2][0] = detinv * (a(2, 1) * (a(3, 2) * a(4, 4) - a(3, 4) * a(4, 2)) + a(2, 2) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4)) + a(2, 4) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1)));
  B.m[3][0] = detinv * (a(2, 1) * (a(3, 3) * a(4, 2) - a(3, 2) * a(4, 3)) + a(2, 2) * (a(3, 1) * a(4, 3) - a(3, 3) * a(4, 1)) + a(2, 3) * (a(3, 2) * a(4, 1) - a(3, 1) * a(4, 2)));
  B.m[0][1] = detinv * (a(1, 2) * (a(3, 4) * a(4, 3) - a(3, 3) * a(4, 4)) + a(1, 3) * (a(3, 2) * a(4, 4) - a(3, 4) * a(4, 2)) + a(1, 4) * (a(3, 3) * a(4, 2) - a(3, 2) * a(4, 3)));
  B.m[1][1] = detinv * (a(1, 1) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3)) + a(1, 3) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4)) + a(1, 4) * (a(3, 1) * a(4, 3) - a(3, 3) * a(4, 1)));
  B.m[2][1] = detinv * (a(1, 1) * (a(3, 4) * a(4, 2) - a(3, 2) * a(4, 4)) + a(1, 2) * (a(3, 1) * a(4, 4) - a(3, 4) * a(4, 1)) + a(1, 4) * (a(3, 2) * a(4, 1) - a(3, 1) * a(4, 2)));
  B.m[3][1] = detinv * (a(1, 1) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2)) + a(1, 2) * (a(3, 3) * a(4, 1) - a(3, 1) * a(4, 3)) + a(1, 3) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1)));
  B.m[0][2] = detinv * (a(1, 2) * (a(2, 3) * a(4, 4) - a(2, 4) * a(4, 3)) + a(1, 3) * (a(2, 4) * a(4, 2) - a(2, 2) * a(4, 4)) + a(1, 4) * (a(2, 2) * a(4, 3) - a(2, 3) * a(4, 2)));
  B.m[1][2] = detinv * (a(1, 1) * (a(2, 4) * a(4, 3) - a(2, 3) * a(4, 4)) + a(1, 3) * (a(2, 1) * a(4, 4) - a(2, 4) * a(4, 1)) + a(1, 4) * (a(2, 3) * a(4, 1) - a(2, 1) * a(4, 3)));
  B.m[2][2] = detinv * (a(1, 1) * (a(2, 2) * a(4, 4) - a(2, 4) * a(4, 2)) + a(1, 2) * (a(2, 4) * a(4, 1) - a(2, 1) * a(4, 4)) + a(1, 4) * (a(2, 1) * a(4, 2) - a(2, 2) * a(4, 1)));
  B.m[3][2] = detinv * (a(1, 1) * (a(2, 3) * a(4, 2) - a(2, 2) * a(4, 3)) + a(1, 2) * (a(2, 1) * a(4, 3) - a(2, 3) * a(4, 1)) + a(1, 3) * (a(2, 2) * a(4, 1) - a(2, 1) * a(4, 2)));
  B.m[0][3] = detinv * (a(1, 2) * (a(2, 4) * a(3, 3) - a(2, 3) * a(3, 4)) + a(1, 3) * (a(2, 2) * a(3, 4) - a(2, 4) * a(3, 2)) + a(1, 4) * (a(2, 3) * a(3, 2) - a(2, 2) * a(3, 3)));
  B.m[1][3] = detinv * (a(1, 1) * (a(2, 3) * a(3, 4) - a(2, 4) * a(3, 3)) + a(1, 3) * (a(2, 4) * a(3, 1) - a(2, 1) * a(3, 4)) + a(1, 4) * (a(2, 1) * a(3, 3) - a(2, 3) * a(3, 1)));
  B.m[2][3] = detinv * (a(1, 1) * (a(2, 4) * a(3, 2) - a(2, 2) * a(3, 4)) + a(1, 2) * (a(2, 1) * a(3, 4) - a(2, 4) * a(3, 1)) + a(1, 4) * (a(2, 2) * a(3, 1) - a(2, 1) * a(3, 2)));
  B.m[3][3] = detinv * (a(1, 1) * (a(2, 2) * a(3, 3) - a(2, 3) * a(3, 2)) + a(1, 2) * (a(2, 3) * a(3, 1) - a(2, 1) * a(3, 3)) + a(1, 3) * (a(2, 1) * a(3, 2) - a(2, 2) * a(3, 1)));
  return B;
}


// matmul(A, B) for 4x4 (Fortran intrinsic): C(i,j) = sum_k A(i,k)*B(k,j), k ascending.
inline M4 matmul(const M4& A, const M4& B) {
  M4 C{};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s = s + A.m[i][k] * B.m[k][j];
      C.m[i][j] = s;
    }
  return C;
}

struct V3h {
  double x, y, z;
};
inline double dot(V3h a, V3h b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // vector_class.f90:279-290
inline V3h cross(V3h a, V3h b) {                                              // vector_class.f90:306-318
  return V3h{a.y * b.z - a.z * b.y, -a.x * b.z + a.z * b.x, a.x * b.y - a.y * b.x};
}
inline double length(V3h a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  // :405-411
inline V3h magnitude(V3h a) {                                                          // :392-402
  const double t = length(a);
  return V3h{a.x / t, a.y / t, a.z / t};
}
inline bool veq(V3h a, V3h b) { return a.x == b.x && a.y == b.y && a.z == b.z; }  // vec_equal_vec :131-146
inline V3h vabs(V3h a) { return V3h{std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)}; }

// rotationAlign(a, b), sdfHelpers.f90:114-140: I + [v]x + [v]x^2 / (1 + a.b), v = a x b.
inline M4 rotation_align(V3h a, V3h b) {
  const V3h v = cross(a, b);
  const double c = dot(a, b);
  const double k = 1.0 / (1.0 + c);
  M4 vx{};  // columns (0,-vz,vy,0) (vz,0,-vx,0) (-vy,vx,0,0) (0,0,0,0)
  vx.m[0][0] = 0.0;        vx.m[1][0] = -1.0 * v.z; vx.m[2][0] = v.y;        vx.m[3][0] = 0.0;
  vx.m[0][1] = v.z;        vx.m[1][1] = 0.0;        vx.m[2][1] = -1.0 * v.x; vx.m[3][1] = 0.0;
  vx.m[0][2] = -1.0 * v.y; vx.m[1][2] = v.x;        vx.m[2][2] = 0.0;        vx.m[3][2] = 0.0;
  const M4 vx2 = matmul(vx, vx);
  const M4 I = identity();
  M4 r{};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) r.m[i][j] = (I.m[i][j] + vx.m[i][j]) + vx2.m[i][j] * k;
  return r;
}

// Column-major copy (Fortran t(r,c) -> out[(c-1)*4 + (r-1)]).
inline void to_colmajor(const M4& a, double* out) {
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) out[c * 4 + r] = a.m[r][c];
}

}  // namespace mat
}  // namespace smcrt
