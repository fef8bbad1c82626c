// osc_kin_device.hpp -- the rigid-body kinematics front end's device code (SURVEY.md §8(f) row 1;
// formulation: osc_kinematics.hip's header): the model tables (KinDev), the per-env LDS layout and
// the per-stage arithmetic, shared by osc_kinematics_kernel (four envs per wave) and the fused
// joint-state tick (osc_setup.hpp, setup_env<D, true>: one env per wave, the kinematics in the
// assembly kernel's prologue, M, C, J, b straight into its LDS).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "osc_kinematics.h"

namespace osc_kin {

constexpr int kBodyStride = 40;   // doubles of per-body LDS state (see the B_* offsets)
constexpr int kDofStride = 12;    // S (6) | F = Ic S (6)

// per-body LDS state offsets
constexpr int B_R = 0, B_X = 9, B_W = 12, B_VO = 15, B_AL = 18, B_AO = 21, B_M = 24, B_H = 25,
              B_IO = 28, B_F = 34;   // IO: xx yy zz xy xz yz;  F: (n, f) total force

// Device-resident model tables (derived on the host from osc_kin_desc).
struct alignas(16) KinDev {   // alignas: sizeof % 16 == 0 (16-byte LDS staging)
  int32_t nbody, nq, nv, nsite, ndepth;
  int32_t parent[OSC_KIN_MAX_BODIES];
  int32_t jtype[OSC_KIN_MAX_BODIES];
  int32_t qadr[OSC_KIN_MAX_BODIES];
  int32_t dadr[OSC_KIN_MAX_BODIES];
  int32_t depth[OSC_KIN_MAX_BODIES];
  int32_t first_child[OSC_KIN_MAX_BODIES];
  int32_t next_sibling[OSC_KIN_MAX_BODIES];
  uint32_t anc[OSC_KIN_MAX_BODIES];          // ancestor-or-self body mask
  int32_t dof_body[OSC_KIN_MAX_DOFS];
  int32_t site_body[OSC_KIN_MAX_SITES];      // body carrying the site point
  int32_t site_jac[OSC_KIN_MAX_SITES];       // Jacobian body (mj_jac's body argument)
  uint32_t dof_relmask[OSC_KIN_MAX_DOFS];    // dofs j with M_ij structurally non-zero
  double dof_arm[OSC_KIN_MAX_DOFS];          // dof_armature
  uint32_t site_dofmask[OSC_KIN_MAX_SITES];  // ancestor dofs of the site's Jacobian body
  double gravity[3];
  double rq[OSC_KIN_MAX_BODIES][9];          // body_quat as a rotation (row-major)
  double pos[OSC_KIN_MAX_BODIES][3];
  double axis[OSC_KIN_MAX_BODIES][3];        // unit
  double jpos[OSC_KIN_MAX_BODIES][3];
  double arm[OSC_KIN_MAX_BODIES];
  double mass[OSC_KIN_MAX_BODIES];
  double ipos[OSC_KIN_MAX_BODIES][3];
  double ib[OSC_KIN_MAX_BODIES][6];          // body-frame inertia about the COM
  double site_pos[OSC_KIN_MAX_SITES][3];
};

constexpr int even(int a) { return (a + 1) & ~1; }

struct EnvLayout {   // per-env LDS layout in doubles
  int q, body, dof, site, size;
  __host__ __device__ EnvLayout(int nq, int nv, int nb, int ns) {
    q = 0;
    body = even(nq + nv);
    dof = body + kBodyStride * nb;
    site = dof + kDofStride * nv;
    size = even(site + 3 * ns);
  }
};

__device__ __forceinline__ void wave_sync() {   // one wavefront per workgroup
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void cross(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// (n, f) = I (w, v) with I = (m, h, IO)
__device__ __forceinline__ void inertia_mul(double m, const double* h, const double* IO,
                                            const double* w, const double* v, double* n,
                                            double* f) {
  double hv[3], hw[3];
  cross(h, v, hv);
  cross(h, w, hw);
  n[0] = IO[0] * w[0] + IO[3] * w[1] + IO[4] * w[2] + hv[0];
  n[1] = IO[3] * w[0] + IO[1] * w[1] + IO[5] * w[2] + hv[1];
  n[2] = IO[4] * w[0] + IO[5] * w[1] + IO[2] * w[2] + hv[2];
  for (int k = 0; k < 3; ++k) f[k] = m * v[k] - hw[k];
}

// Forward pass for body b (its parent's state is final): frame, velocity, bias acceleration,
// spatial inertia and the body's own RNEA force.  Writes the body's LDS state.
static __device__ void body_forward(const KinDev* K, double* E, const EnvLayout& lay,
                             int b, double s, double c) {
  double R[9], x[3], w[3], vo[3], al[3], ao[3];
  const int jt = K->jtype[b];
  const double* q = E + lay.q;
  const double* qd = E + lay.q + K->nq;
  if (jt == OSC_KIN_JOINT_FREE) {
    const int qa = K->qadr[b], da = K->dadr[b];
    x[0] = q[qa];
    x[1] = q[qa + 1];
    x[2] = q[qa + 2];
    double qw = q[qa + 3], qx = q[qa + 4], qy = q[qa + 5], qz = q[qa + 6];
    const double inv = 1.0 / sqrt(qw * qw + qx * qx + qy * qy + qz * qz);
    qw *= inv; qx *= inv; qy *= inv; qz *= inv;
    R[0] = 1 - 2 * (qy * qy + qz * qz); R[1] = 2 * (qx * qy - qw * qz); R[2] = 2 * (qx * qz + qw * qy);
    R[3] = 2 * (qx * qy + qw * qz); R[4] = 1 - 2 * (qx * qx + qz * qz); R[5] = 2 * (qy * qz - qw * qx);
    R[6] = 2 * (qx * qz - qw * qy); R[7] = 2 * (qy * qz + qw * qx); R[8] = 1 - 2 * (qx * qx + qy * qy);
    const double v[3] = {qd[da], qd[da + 1], qd[da + 2]};
    const double wl[3] = {qd[da + 3], qd[da + 4], qd[da + 5]};
    for (int i = 0; i < 3; ++i) w[i] = R[3 * i] * wl[0] + R[3 * i + 1] * wl[1] + R[3 * i + 2] * wl[2];
    double xw[3];
    cross(x, w, xw);
    for (int i = 0; i < 3; ++i) {
      vo[i] = v[i] + xw[i];     // v_O = v - w x x
      al[i] = 0.0;
    }
    cross(v, w, ao);            // a_O = v x w  (the body origin itself does not accelerate)
  } else {
    const int p = K->parent[b];
    double pR[9], px[3], pw[3], pvo[3], pal[3], pao[3];
    if (p >= 0) {
      const double* P = E + lay.body + kBodyStride * p;
      for (int i = 0; i < 9; ++i) pR[i] = P[B_R + i];
      for (int i = 0; i < 3; ++i) {
        px[i] = P[B_X + i]; pw[i] = P[B_W + i]; pvo[i] = P[B_VO + i];
        pal[i] = P[B_AL + i]; pao[i] = P[B_AO + i];
      }
    } else {
      for (int i = 0; i < 9; ++i) pR[i] = (i % 4 == 0) ? 1.0 : 0.0;
      for (int i = 0; i < 3; ++i) px[i] = pw[i] = pvo[i] = pal[i] = pao[i] = 0.0;
    }
    const double* rq = K->rq[b];
    const double* bp = K->pos[b];
    double Rb[9];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j)
        Rb[3 * i + j] = pR[3 * i] * rq[j] + pR[3 * i + 1] * rq[3 + j] + pR[3 * i + 2] * rq[6 + j];
      x[i] = px[i] + pR[3 * i] * bp[0] + pR[3 * i + 1] * bp[1] + pR[3 * i + 2] * bp[2];
    }
    if (jt == OSC_KIN_JOINT_HINGE || jt == OSC_KIN_JOINT_BALL) {
      // rotation about the anchor: R = Rb Ra, the anchor stays put
      const double* jp = K->jpos[b];
      double anc[3], Ra[9];
      for (int i = 0; i < 3; ++i)
        anc[i] = x[i] + Rb[3 * i] * jp[0] + Rb[3 * i + 1] * jp[1] + Rb[3 * i + 2] * jp[2];
      if (jt == OSC_KIN_JOINT_HINGE) {
        // Rodrigues in the body frame: Raa = c I + s [u]x + (1 - c) u u'
        const double* u = K->axis[b];
        const double t = 1.0 - c;
        Ra[0] = c + t * u[0] * u[0]; Ra[1] = t * u[0] * u[1] - s * u[2]; Ra[2] = t * u[0] * u[2] + s * u[1];
        Ra[3] = t * u[0] * u[1] + s * u[2]; Ra[4] = c + t * u[1] * u[1]; Ra[5] = t * u[1] * u[2] - s * u[0];
        Ra[6] = t * u[0] * u[2] - s * u[1]; Ra[7] = t * u[1] * u[2] + s * u[0]; Ra[8] = c + t * u[2] * u[2];
      } else {   // ball: qpos = unit quaternion of the body relative to its parent frame
        const int qa = K->qadr[b];
        double qw = q[qa], qx = q[qa + 1], qy = q[qa + 2], qz = q[qa + 3];
        const double inv = 1.0 / sqrt(qw * qw + qx * qx + qy * qy + qz * qz);
        qw *= inv; qx *= inv; qy *= inv; qz *= inv;
        Ra[0] = 1 - 2 * (qy * qy + qz * qz); Ra[1] = 2 * (qx * qy - qw * qz); Ra[2] = 2 * (qx * qz + qw * qy);
        Ra[3] = 2 * (qx * qy + qw * qz); Ra[4] = 1 - 2 * (qx * qx + qz * qz); Ra[5] = 2 * (qy * qz - qw * qx);
        Ra[6] = 2 * (qx * qz - qw * qy); Ra[7] = 2 * (qy * qz + qw * qx); Ra[8] = 1 - 2 * (qx * qx + qy * qy);
      }
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
          R[3 * i + j] = Rb[3 * i] * Ra[j] + Rb[3 * i + 1] * Ra[3 + j] + Rb[3 * i + 2] * Ra[6 + j];
      for (int i = 0; i < 3; ++i)
        x[i] = anc[i] - (R[3 * i] * jp[0] + R[3 * i + 1] * jp[1] + R[3 * i + 2] * jp[2]);
      // joint motion (wj, vj) = S qd: hinge S = (a, anc x a) with a = Rb u (fixed in the parent);
      // ball S = (R e_k, anc x R e_k), qd = body-frame angular velocity.  Either S is fixed in the
      // body, so dS/dt qd = v_b x (S qd) = v_p x (S qd): the same bias terms as the hinge.
      double wj[3], vj[3];
      if (jt == OSC_KIN_JOINT_HINGE) {
        const double* u = K->axis[b];
        const double qv = qd[K->dadr[b]];
        for (int i = 0; i < 3; ++i)
          wj[i] = (Rb[3 * i] * u[0] + Rb[3 * i + 1] * u[1] + Rb[3 * i + 2] * u[2]) * qv;
      } else {
        const int da = K->dadr[b];
        const double wl[3] = {qd[da], qd[da + 1], qd[da + 2]};
        for (int i = 0; i < 3; ++i) wj[i] = R[3 * i] * wl[0] + R[3 * i + 1] * wl[1] + R[3 * i + 2] * wl[2];
      }
      cross(anc, wj, vj);
      for (int i = 0; i < 3; ++i) {
        w[i] = pw[i] + wj[i];
        vo[i] = pvo[i] + vj[i];
      }
      double c1[3], c2[3], c3[3];
      cross(pw, wj, c1);
      cross(pw, vj, c2);
      cross(pvo, wj, c3);
      for (int i = 0; i < 3; ++i) {
        al[i] = pal[i] + c1[i];
        ao[i] = pao[i] + c2[i] + c3[i];
      }
    } else if (jt == OSC_KIN_JOINT_SLIDE) {
      // translation along a = Rb u (fixed in the parent): S = (0, a), bias v_p x (0, a qd)
      const double* u = K->axis[b];
      const double qv = q[K->qadr[b]], qdv = qd[K->dadr[b]];
      double vj[3], c2[3];
      for (int i = 0; i < 3; ++i) {
        const double a = Rb[3 * i] * u[0] + Rb[3 * i + 1] * u[1] + Rb[3 * i + 2] * u[2];
        x[i] += a * qv;
        vj[i] = a * qdv;
      }
      for (int i = 0; i < 9; ++i) R[i] = Rb[i];
      cross(pw, vj, c2);
      for (int i = 0; i < 3; ++i) {
        w[i] = pw[i]; vo[i] = pvo[i] + vj[i]; al[i] = pal[i]; ao[i] = pao[i] + c2[i];
      }
    } else {   // welded to the parent
      for (int i = 0; i < 9; ++i) R[i] = Rb[i];
      for (int i = 0; i < 3; ++i) {
        w[i] = pw[i]; vo[i] = pvo[i]; al[i] = pal[i]; ao[i] = pao[i];
      }
    }
  }
  double* B = E + lay.body + kBodyStride * b;
  for (int i = 0; i < 9; ++i) B[B_R + i] = R[i];
  for (int i = 0; i < 3; ++i) {
    B[B_X + i] = x[i]; B[B_W + i] = w[i]; B[B_VO + i] = vo[i];
    B[B_AL + i] = al[i]; B[B_AO + i] = ao[i];
  }
}

// Body b's spatial inertia about the world origin and its own RNEA force, once its frame and
// motion are in LDS (all bodies in parallel, after the level-by-level pass).
static __device__ void body_dynamics(const KinDev* K, double* E, const EnvLayout& lay, int b) {
  double* B = E + lay.body + kBodyStride * b;
  double R[9], x[3], w[3], vo[3], al[3], ao[3];
  for (int i = 0; i < 9; ++i) R[i] = B[B_R + i];
  for (int i = 0; i < 3; ++i) {
    x[i] = B[B_X + i]; w[i] = B[B_W + i]; vo[i] = B[B_VO + i];
    al[i] = B[B_AL + i]; ao[i] = B[B_AO + i];
  }
  // IO = R Ib R' + m (|c|^2 I - c c'), h = m c
  const double m = K->mass[b];
  const double* ip = K->ipos[b];
  const double* ib = K->ib[b];
  double c[3];
  for (int i = 0; i < 3; ++i) c[i] = x[i] + R[3 * i] * ip[0] + R[3 * i + 1] * ip[1] + R[3 * i + 2] * ip[2];
  const double Ibf[9] = {ib[0], ib[3], ib[4], ib[3], ib[1], ib[5], ib[4], ib[5], ib[2]};
  double RI[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      RI[3 * i + j] = R[3 * i] * Ibf[j] + R[3 * i + 1] * Ibf[3 + j] + R[3 * i + 2] * Ibf[6 + j];
  auto rir = [&](int i, int j) {
    return RI[3 * i] * R[3 * j] + RI[3 * i + 1] * R[3 * j + 1] + RI[3 * i + 2] * R[3 * j + 2];
  };
  const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  double IO[6], h[3];
  IO[0] = rir(0, 0) + m * (cc - c[0] * c[0]);
  IO[1] = rir(1, 1) + m * (cc - c[1] * c[1]);
  IO[2] = rir(2, 2) + m * (cc - c[2] * c[2]);
  IO[3] = rir(0, 1) - m * c[0] * c[1];
  IO[4] = rir(0, 2) - m * c[0] * c[2];
  IO[5] = rir(1, 2) - m * c[1] * c[2];
  for (int i = 0; i < 3; ++i) h[i] = m * c[i];
  // own RNEA force: f = I (al, a_O - g) + v x* (I v)
  double ag[3];
  for (int i = 0; i < 3; ++i) ag[i] = ao[i] - K->gravity[i];
  double n1[3], f1[3], ln[3], lf[3];
  inertia_mul(m, h, IO, al, ag, n1, f1);
  inertia_mul(m, h, IO, w, vo, ln, lf);
  double t1[3], t2[3], t3[3];
  cross(w, ln, t1);
  cross(vo, lf, t2);
  cross(w, lf, t3);
  for (int i = 0; i < 3; ++i) {
    B[B_H + i] = h[i];
    B[B_F + i] = n1[i] + t1[i] + t2[i];
    B[B_F + 3 + i] = f1[i] + t3[i];
  }
  B[B_M] = m;
  for (int i = 0; i < 6; ++i) B[B_IO + i] = IO[i];
}

// ---- per-stage helpers shared by osc_kinematics_kernel (four envs per wave, 16 lanes each) and
// the fused joint-state setup kernel (osc_setup.hpp: one env per wave, 64 lanes): the same
// arithmetic in both, so the fused tick's M, C, J, b are bitwise the kinematics kernel's ----

// Stage 1, forward pass level by level (lane = body l; lanes past nbody idle).  Every lane of the
// wave calls it (wave barriers inside).  Every hinge's sin / cos up front (all lanes at once), so
// the level loop -- whose body executes once per level -- carries no libm call; the inertia /
// force work, which needs no parent data, runs once for all bodies after it.
__device__ __forceinline__ void kin_forward(const KinDev* K, double* E, const EnvLayout& lay,
                                            int l) {
  const int nb = K->nbody, nd = K->ndepth;
  const int my_depth = (l < nb) ? K->depth[l] : -1;
  double sn = 0.0, cs = 1.0;
  if (l < nb && K->jtype[l] == OSC_KIN_JOINT_HINGE) sincos(E[lay.q + K->qadr[l]], &sn, &cs);
  for (int L = 0; L < nd; ++L) {
    if (my_depth == L) body_forward(K, E, lay, l, sn, cs);
    wave_sync();
  }
  if (l < nb) body_dynamics(K, E, lay, l);
  wave_sync();
}

// Stage 2, backward pass: subtree composite inertia and force (lane = body l).
__device__ __forceinline__ void kin_backward(const KinDev* K, double* E, const EnvLayout& lay,
                                             int l) {
  const int nb = K->nbody, nd = K->ndepth;
  const int my_depth = (l < nb) ? K->depth[l] : -1;
  for (int L = nd - 2; L >= 0; --L) {
    if (my_depth == L) {
      double* B = E + lay.body + kBodyStride * l;
      double acc[10 + 6];
      for (int i = 0; i < 10; ++i) acc[i] = B[B_M + i];
      for (int i = 0; i < 6; ++i) acc[10 + i] = B[B_F + i];
      for (int ch = K->first_child[l]; ch >= 0; ch = K->next_sibling[ch]) {
        const double* Cb = E + lay.body + kBodyStride * ch;
        for (int i = 0; i < 10; ++i) acc[i] += Cb[B_M + i];
        for (int i = 0; i < 6; ++i) acc[10 + i] += Cb[B_F + i];
      }
      for (int i = 0; i < 10; ++i) B[B_M + i] = acc[i];
      for (int i = 0; i < 6; ++i) B[B_F + i] = acc[10 + i];
    }
    wave_sync();
  }
}

// Stage 3 for dof d: motion subspace S and F = Ic S into the dof's LDS slot; returns C_d = S . f.
__device__ __forceinline__ double kin_dof(const KinDev* K, double* E, const EnvLayout& lay,
                                          int d) {
  const int bb = K->dof_body[d];
  const double* B = E + lay.body + kBodyStride * bb;
  double S[6];
  const int k = d - K->dadr[bb];
  if (K->jtype[bb] == OSC_KIN_JOINT_FREE) {
    if (k < 3) {
      S[0] = S[1] = S[2] = 0.0;
      for (int i = 0; i < 3; ++i) S[3 + i] = (i == k) ? 1.0 : 0.0;
    } else {
      const double a[3] = {B[B_R + k - 3], B[B_R + 3 + k - 3], B[B_R + 6 + k - 3]};
      const double xo[3] = {B[B_X], B[B_X + 1], B[B_X + 2]};
      S[0] = a[0]; S[1] = a[1]; S[2] = a[2];
      cross(xo, a, S + 3);
    }
  } else if (K->jtype[bb] == OSC_KIN_JOINT_SLIDE) {   // (0, a), a = R u
    const double* u = K->axis[bb];
    S[0] = S[1] = S[2] = 0.0;
    for (int i = 0; i < 3; ++i)
      S[3 + i] = B[B_R + 3 * i] * u[0] + B[B_R + 3 * i + 1] * u[1] + B[B_R + 3 * i + 2] * u[2];
  } else {   // hinge (a = R u: the axis is invariant under its own rotation) or ball (a = R e_k)
    const double* u = K->axis[bb];
    const double* jp = K->jpos[bb];
    const bool ball = K->jtype[bb] == OSC_KIN_JOINT_BALL;
    double a[3], pa[3];
    for (int i = 0; i < 3; ++i) {
      a[i] = ball ? B[B_R + 3 * i + k]
                  : B[B_R + 3 * i] * u[0] + B[B_R + 3 * i + 1] * u[1] + B[B_R + 3 * i + 2] * u[2];
      pa[i] = B[B_X + i] + B[B_R + 3 * i] * jp[0] + B[B_R + 3 * i + 1] * jp[1] +
              B[B_R + 3 * i + 2] * jp[2];
    }
    S[0] = a[0]; S[1] = a[1]; S[2] = a[2];
    cross(pa, a, S + 3);
  }
  double F[6];
  inertia_mul(B[B_M], B + B_H, B + B_IO, S, S + 3, F, F + 3);
  double* Dd = E + lay.dof + kDofStride * d;
  for (int i = 0; i < 6; ++i) {
    Dd[i] = S[i];
    Dd[6 + i] = F[i];
  }
  double cd = 0.0;
  for (int i = 0; i < 6; ++i) cd = fma(S[i], B[B_F + i], cd);
  return cd;
}

// Stage 4 for site k: its world position into the site's LDS slot; its J-dot qvel rows,
// translational bp (rows 3k..3k+2 of b) and rotational br (rows 3ns+3k..).
__device__ __forceinline__ void kin_site(const KinDev* K, double* E, const EnvLayout& lay, int k,
                                         double* bp, double* br) {
  const double* Bp = E + lay.body + kBodyStride * K->site_body[k];   // point's body
  const double* B = E + lay.body + kBodyStride * K->site_jac[k];      // Jacobian body
  const double* sp = K->site_pos[k];
  double xk[3];
  for (int i = 0; i < 3; ++i)
    xk[i] = Bp[B_X + i] + Bp[B_R + 3 * i] * sp[0] + Bp[B_R + 3 * i + 1] * sp[1] +
            Bp[B_R + 3 * i + 2] * sp[2];
  double* Xs = E + lay.site + 3 * k;
  for (int i = 0; i < 3; ++i) Xs[i] = xk[i];
  const double w[3] = {B[B_W], B[B_W + 1], B[B_W + 2]};
  const double al[3] = {B[B_AL], B[B_AL + 1], B[B_AL + 2]};
  double wx[3], alx[3], vx[3], wvx[3];
  cross(w, xk, wx);
  cross(al, xk, alx);
  for (int i = 0; i < 3; ++i) vx[i] = B[B_VO + i] + wx[i];
  cross(w, vx, wvx);
  for (int i = 0; i < 3; ++i) {
    bp[i] = B[B_AO + i] + alx[i] + wvx[i];
    br[i] = al[i];
  }
}

// Stage 5, M_ij for row i (S_i, F_i) and column j (S_j, F_j): M_ij = S_lo . (Ic S_hi) for related
// dofs (lo = min(i, j)), + armature on the diagonal (branch-free).
__device__ __forceinline__ double kin_m_entry(uint32_t rel, double arm, int i, int j,
                                              const double* Si, const double* Fi,
                                              const double* Sj, const double* Fj) {
  double up = 0.0, lo = 0.0;
  for (int t = 0; t < 6; ++t) {
    up = fma(Si[t], Fj[t], up);
    lo = fma(Sj[t], Fi[t], lo);
  }
  const double v = (i <= j ? up : lo) + (i == j ? arm : 0.0);
  return ((rel >> j) & 1u) ? v : 0.0;
}

// Stage 6, column c (motion subspace S) of site k at xk: Jp = S.v + S.w x x_k, Jr = S.w when c is
// an ancestor dof of the site's Jacobian body (r), else zero.
__device__ __forceinline__ void kin_j_col(bool r, const double* S, const double* xk, double* jp,
                                          double* jr) {
  double wx[3];
  cross(S, xk, wx);
  for (int t = 0; t < 3; ++t) {
    jp[t] = r ? S[3 + t] + wx[t] : 0.0;
    jr[t] = r ? S[t] : 0.0;
  }
}

}  // namespace osc_kin
