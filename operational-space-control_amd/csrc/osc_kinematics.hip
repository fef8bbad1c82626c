// osc_kinematics.hip -- batched floating-base rigid-body kinematics for gfx950 (MI355X): the
// GPU front end of the OSC solve (C-ABI in include/osc_kinematics.h).
//
// Replaces, per environment, what the reference asks MuJoCo for every tick (paths relative to
// the reference's operational-space-control/):
//   update_mj_data   unitree_go2/operational_space_controller.h:350-374
//   update_osc_data  unitree_go2/operational_space_controller.h:376-455
//     M = mj_fullM (:380), C = qfrc_bias (:383), J = [Jp_0..; Jr_0..] from mj_jac per site
//     (:401-429), b = [Jpd; Jrd] qvel from mj_jacDot (:430-434).
//
// Formulation: spatial vectors in WORLD coordinates about the world origin (Featherstone's
// CRBA / RNEA without any frame transforms between bodies).  For every body b:
//   v_b = (w, v_O)      spatial velocity (angular velocity, velocity of the world-origin point)
//   a_b = (al, a_O)     spatial bias acceleration at zero joint acceleration
//   I_b = (m, h = m c, I_O)   spatial inertia about the origin; I (w, v) = (I_O w + h x v,
//                             m v - h x w)
// A hinge dof has S = (a, p x a) (axis a through anchor p), a slide S = (0, a), a ball's three
// dofs (R e_k, p x R e_k) (body axes through its anchor); a free joint's translational dofs
// are (0, e_k) (world axes) and its rotational dofs (R e_k, x x R e_k) (body axes through the
// body origin: MuJoCo's body-frame angular qvel).  Since S of a hinge / slide is fixed in its
// parent (a ball's in its body, and v_b x S qd = v_p x S qd), a_b = a_p + v_p x (S qd); the free
// root has a = (0, v x w).
//   qfrc_bias: f_b = I_b (a_b - (0, g)) + v_b x* I_b v_b, summed over subtrees, C_d = S_d . f.
//   mj_fullM:  M_ij = S_i . (Ic_{body(j)} S_j) for body(i) an ancestor of body(j) (Ic =
//              subtree composite inertia), + armature on the diagonal.
//   mj_jac:    column d of a point x on body k (d an ancestor dof): Jr = S_d.w,
//              Jp = S_d.v + S_d.w x x.   mj_jacDot qvel: classical acceleration of x at zero
//              joint acceleration, a_O + al x x + w x (v_O + w x x), and al.
// The CPU oracle (oracle/kinematics.py) computes the same quantities a different way (COM
// Jacobians, Kane's method), pinned by finite-difference and energy identities.
//
// Mapping: FOUR environments per 64-lane wavefront, one 16-lane row each (the IPM kernel's
// layout).  Tree recursions run level by level with lane = body (trees are shallow: Go2 4
// levels, WaLTER 3); the dof, site and dense output stages run with lane = dof / site / output
// element, so the M and J rows leave as 128-byte coalesced stores.  Per-env state lives in
// LDS (6.3 KB Go2, 5.1 KB WaLTER), sized at launch from the model.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <new>
#include <sstream>
#include <string>
#include <vector>

#include <dlfcn.h>

#include "osc_batch.h"
#include "osc_kin_device.hpp"
#include "osc_kinematics.h"
#include "osc_qpos.hpp"

namespace {

using namespace osc_kin;

constexpr int kWave = 64;
constexpr int kRow = 16;
constexpr int kEnvPerWave = kWave / kRow;
// Diagnostic builds only (tools/kin_ablate.sh): -DOSC_KIN_STOP=k ends the kernel before stage k.
#ifdef OSC_KIN_STOP
#define KIN_STOP(k) do { if ((k) == OSC_KIN_STOP) return; } while (0)
#else
#define KIN_STOP(k) do {} while (0)
#endif

__global__ __launch_bounds__(kWave) void osc_kinematics_kernel(
    const KinDev* __restrict__ Kg, int nenv, const double* __restrict__ qpos,
    const double* __restrict__ qvel, double* __restrict__ gM, double* __restrict__ gC,
    double* __restrict__ gJ, double* __restrict__ gb, double* __restrict__ gx) {
  extern __shared__ __attribute__((aligned(16))) double kin_sm[];
  // The model tables are indexed per lane (body / dof / site differ across lanes), so they are
  // staged into LDS once per workgroup: ~64-cycle LDS reads instead of dependent L2 round trips
  // in every output-element iteration.
  __shared__ __attribute__((aligned(16))) KinDev sK;
  {
    static_assert(sizeof(KinDev) % 16 == 0, "16-byte staging of the model tables");
    const uint4* src = reinterpret_cast<const uint4*>(Kg);
    uint4* dst = reinterpret_cast<uint4*>(&sK);
    for (int i = threadIdx.x; i < static_cast<int>(sizeof(KinDev) / 16); i += kWave) dst[i] = src[i];
  }
  wave_sync();
  const KinDev* K = &sK;
  const int lane = threadIdx.x;
  const int row = lane / kRow, l = lane % kRow;
  const int env_raw = blockIdx.x * kEnvPerWave + row;
  const bool valid = env_raw < nenv;
  const int env = valid ? env_raw : nenv - 1;   // tail rows recompute the last env, store nothing
  const int nq = Kg->nq, nv = Kg->nv, nb = Kg->nbody, ns = Kg->nsite;
  const EnvLayout lay(nq, nv, nb, ns);
  double* E = kin_sm + row * lay.size;

  // ---- stage 0: qpos | qvel -> LDS --------------------------------------------------------
  for (int i = l; i < nq; i += kRow) E[lay.q + i] = qpos[static_cast<size_t>(env) * nq + i];
  for (int i = l; i < nv; i += kRow) E[lay.q + nq + i] = qvel[static_cast<size_t>(env) * nv + i];
  wave_sync();

  KIN_STOP(0);
  // ---- stage 1: forward pass, level by level (lane = body) --------------------------------
  kin_forward(K, E, lay, l);

  KIN_STOP(1);
  // ---- stage 2: backward pass: subtree composite inertia and force ------------------------
  kin_backward(K, E, lay, l);

  KIN_STOP(2);
  // ---- stage 3: dofs (lane = dof): motion subspace S, F = Ic S, C = S . f -----------------
  for (int d = l; d < nv; d += kRow) {
    const double cd = kin_dof(K, E, lay, d);
    if (valid) gC[static_cast<size_t>(env) * nv + d] = cd;
  }

  KIN_STOP(3);
  // ---- stage 4: sites (lane = site): world position, J-dot qvel ---------------------------
  for (int k = l; k < ns; k += kRow) {
    double bp[3], br[3];
    kin_site(K, E, lay, k, bp, br);
    if (valid) {
      double* bo = gb + static_cast<size_t>(env) * 6 * ns;
      for (int i = 0; i < 3; ++i) {
        bo[3 * k + i] = bp[i];
        bo[3 * ns + 3 * k + i] = br[i];
      }
      if (gx) {
        const double* xs = E + lay.site + 3 * k;
        for (int i = 0; i < 3; ++i) gx[(static_cast<size_t>(env) * ns + k) * 3 + i] = xs[i];
      }
    }
  }
  wave_sync();

  KIN_STOP(4);
  // ---- stage 5: M (lane = columns l, l + 16; uniform loop over rows) -----------------------
  // M_ij = S_lo . (Ic S_hi) for related dofs (lo = min(i, j)); lane j keeps S_j, F_j in
  // registers, row i's S_i, F_i are row-broadcast LDS reads, relations come from per-dof masks
  // (scalar loads).  Every store writes 16 consecutive doubles of one row.
  const int c0 = l, c1 = l + kRow;
  const bool v0 = c0 < nv, v1 = c1 < nv;
  double S0[6], F0[6], S1[6], F1[6];
  {
    const double* D0 = E + lay.dof + kDofStride * (v0 ? c0 : 0);
    const double* D1 = E + lay.dof + kDofStride * (v1 ? c1 : 0);
    for (int t = 0; t < 6; ++t) {
      S0[t] = D0[t]; F0[t] = D0[6 + t];
      S1[t] = D1[t]; F1[t] = D1[6 + t];
    }
  }
  {
    double* Mo = gM + static_cast<size_t>(env) * nv * nv;
    for (int i = 0; i < nv; ++i) {
      const uint32_t rel = K->dof_relmask[i];
      const double arm = K->dof_arm[i];
      const double* Di = E + lay.dof + kDofStride * i;
      double Si[6], Fi[6];
      for (int t = 0; t < 6; ++t) {
        Si[t] = Di[t];
        Fi[t] = Di[6 + t];
      }
      const double m0 = kin_m_entry(rel, arm, i, c0, Si, Fi, S0, F0);
      const double m1 = kin_m_entry(rel, arm, i, c1, Si, Fi, S1, F1);
      if (valid && v0) Mo[i * nv + c0] = m0;
      if (valid && v1) Mo[i * nv + c1] = m1;
    }
  }

  KIN_STOP(5);
  // ---- stage 6: J (lane = columns l, l + 16; uniform loop over sites) ---------------------
  // column c of site k (c an ancestor dof of the site's body): Jr = S_c.w, Jp = S_c.v +
  // S_c.w x x_k; rows 3k..3k+2 (Jp) and 3ns+3k.. (Jr).
  {
    double* Jo = gJ + static_cast<size_t>(env) * 6 * ns * nv;
    for (int k = 0; k < ns; ++k) {
      const uint32_t rel = K->site_dofmask[k];
      const double* xs = E + lay.site + 3 * k;
      const double xk[3] = {xs[0], xs[1], xs[2]};
      auto col = [&](int c, bool vc, const double* S) {
        double jp[3], jr[3];
        kin_j_col(vc && ((rel >> c) & 1u), S, xk, jp, jr);
        for (int t = 0; t < 3; ++t) {
          if (valid && vc) {
            Jo[(3 * k + t) * nv + c] = jp[t];
            Jo[(3 * ns + 3 * k + t) * nv + c] = jr[t];
          }
        }
      };
      col(c0, v0, S0);
      col(c1, v1, S1);
    }
  }
}

constexpr int kPackBlock = 256;

// update_mj_data's qpos / qvel packing for a batch of States (osc.h:357-361).
__global__ __launch_bounds__(kPackBlock) void state_to_qpos_kernel(
    int nenv, int nu, const double* __restrict__ rot, const double* __restrict__ lin,
    const double* __restrict__ ang, const double* __restrict__ mpos,
    const double* __restrict__ mvel, double* __restrict__ qpos, double* __restrict__ qvel) {
  const int nq = 7 + nu, nvv = 6 + nu;
  const long long total = static_cast<long long>(nenv) * (nq + nvv);
  for (long long t = static_cast<long long>(blockIdx.x) * kPackBlock + threadIdx.x; t < total;
       t += static_cast<long long>(gridDim.x) * kPackBlock) {
    const long long e = t / (nq + nvv);
    const int i = static_cast<int>(t - e * (nq + nvv));
    if (i < nq) {
      double v;
      if (i < 3) v = 0.0;                       // base position forced to zero (osc.h:358-359)
      else if (i < 7) v = rot[e * 4 + (i - 3)];
      else v = mpos[e * nu + (i - 7)];
      qpos[e * nq + i] = v;
    } else {
      const int k = i - nq;
      double v;
      if (k < 3) v = lin[e * 3 + k];
      else if (k < 6) v = ang[e * 3 + (k - 3)];
      else v = mvel[e * nu + (k - 6)];
      qvel[e * nvv + k] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------

void quat_to_mat(const double* q, double* R) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  const double n = std::sqrt(w * w + x * x + y * y + z * z);
  w /= n; x /= n; y /= n; z /= n;
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}

int build_tables(const osc_kin_desc& d, KinDev* k) {
  std::memset(k, 0, sizeof(*k));
  if (d.nbody < 1 || d.nbody > OSC_KIN_MAX_BODIES || d.nsite < 1 || d.nsite > OSC_KIN_MAX_SITES)
    return OSC_ERR_INVALID_ARGUMENT;
  int nq = 0, nv = 0, ndepth = 0;
  for (int b = 0; b < d.nbody; ++b) {
    const int p = d.parent[b];
    if (p < -1 || p >= b) return OSC_ERR_INVALID_ARGUMENT;   // parents first (MuJoCo order)
    const int jt = d.jnt_type[b];
    if (jt != OSC_KIN_JOINT_NONE && jt != OSC_KIN_JOINT_FREE && jt != OSC_KIN_JOINT_BALL &&
        jt != OSC_KIN_JOINT_SLIDE && jt != OSC_KIN_JOINT_HINGE)
      return OSC_ERR_INVALID_ARGUMENT;
    if (jt == OSC_KIN_JOINT_FREE && p != -1) return OSC_ERR_INVALID_ARGUMENT;
    if (!(d.mass[b] >= 0.0) || !(d.armature[b] >= 0.0)) return OSC_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < 3; ++i)
      if (!(d.inertia[b][i] >= 0.0)) return OSC_ERR_INVALID_ARGUMENT;
    const double qn = std::sqrt(d.quat[b][0] * d.quat[b][0] + d.quat[b][1] * d.quat[b][1] +
                                d.quat[b][2] * d.quat[b][2] + d.quat[b][3] * d.quat[b][3]);
    const double in = std::sqrt(d.iquat[b][0] * d.iquat[b][0] + d.iquat[b][1] * d.iquat[b][1] +
                                d.iquat[b][2] * d.iquat[b][2] + d.iquat[b][3] * d.iquat[b][3]);
    if (!(qn > 0.0) || !(in > 0.0)) return OSC_ERR_INVALID_ARGUMENT;
    k->parent[b] = p;
    k->jtype[b] = jt;
    k->qadr[b] = nq;
    k->dadr[b] = nv;
    k->depth[b] = p < 0 ? 0 : k->depth[p] + 1;
    ndepth = std::max(ndepth, k->depth[b] + 1);
    k->anc[b] = (p < 0 ? 0u : k->anc[p]) | (1u << b);
    k->first_child[b] = -1;
    k->next_sibling[b] = -1;
    int ndof = 0;
    if (jt == OSC_KIN_JOINT_FREE) {
      nq += 7;
      ndof = 6;
    } else if (jt == OSC_KIN_JOINT_BALL) {
      nq += 4;
      ndof = 3;
    } else if (jt == OSC_KIN_JOINT_HINGE || jt == OSC_KIN_JOINT_SLIDE) {
      nq += 1;
      ndof = 1;
      const double an = std::sqrt(d.axis[b][0] * d.axis[b][0] + d.axis[b][1] * d.axis[b][1] +
                                  d.axis[b][2] * d.axis[b][2]);
      if (!(an > 0.0)) return OSC_ERR_INVALID_ARGUMENT;
      for (int i = 0; i < 3; ++i) k->axis[b][i] = d.axis[b][i] / an;
    }
    if (nv + ndof > OSC_KIN_MAX_DOFS) return OSC_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < ndof; ++i) k->dof_body[nv + i] = b;
    nv += ndof;
    quat_to_mat(d.quat[b], k->rq[b]);
    double Ri[9];
    quat_to_mat(d.iquat[b], Ri);
    double Ib[9];   // Ri diag(I) Ri'
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += Ri[3 * i + t] * d.inertia[b][t] * Ri[3 * j + t];
        Ib[3 * i + j] = s;
      }
    k->ib[b][0] = Ib[0]; k->ib[b][1] = Ib[4]; k->ib[b][2] = Ib[8];
    k->ib[b][3] = Ib[1]; k->ib[b][4] = Ib[2]; k->ib[b][5] = Ib[5];
    for (int i = 0; i < 3; ++i) {
      k->pos[b][i] = d.pos[b][i];
      k->jpos[b][i] = d.jnt_pos[b][i];
      k->ipos[b][i] = d.ipos[b][i];
    }
    k->arm[b] = d.armature[b];
    k->mass[b] = d.mass[b];
  }
  if (nv < 1) return OSC_ERR_INVALID_ARGUMENT;
  // child lists in body order (fixed summation order: deterministic results)
  for (int b = d.nbody - 1; b >= 0; --b) {
    const int p = d.parent[b];
    if (p >= 0) {
      k->next_sibling[b] = k->first_child[p];
      k->first_child[p] = b;
    }
  }
  for (int s = 0; s < d.nsite; ++s) {
    if (d.site_body[s] < 0 || d.site_body[s] >= d.nbody) return OSC_ERR_INVALID_ARGUMENT;
    k->site_body[s] = d.site_body[s];
    k->site_jac[s] = d.has_jac_body ? d.site_jac_body[s] : d.site_body[s];
    if (k->site_jac[s] < 0 || k->site_jac[s] >= d.nbody) return OSC_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < 3; ++i) k->site_pos[s][i] = d.site_pos[s][i];
  }
  for (int i = 0; i < 3; ++i) k->gravity[i] = d.gravity[i];
  static_assert(OSC_KIN_MAX_DOFS <= 32, "dof masks are 32-bit");
  for (int i = 0; i < nv; ++i)
    for (int j = 0; j < nv; ++j) {
      const int bi = k->dof_body[i], bj = k->dof_body[j];
      if (((k->anc[bj] >> bi) & 1u) || ((k->anc[bi] >> bj) & 1u)) k->dof_relmask[i] |= 1u << j;
    }
  for (int i = 0; i < nv; ++i) k->dof_arm[i] = k->arm[k->dof_body[i]];
  for (int s = 0; s < d.nsite; ++s)
    for (int j = 0; j < nv; ++j)
      if ((k->anc[k->site_jac[s]] >> k->dof_body[j]) & 1u) k->site_dofmask[s] |= 1u << j;
  k->nbody = d.nbody;
  k->nq = nq;
  k->nv = nv;
  k->nsite = d.nsite;
  k->ndepth = ndepth;
  return OSC_OK;
}

// ---- minimal JSON reader for the <robot>_kinematics.json schema ----------------------------
struct JVal {
  enum Kind { NUL, NUM, STR, ARR, OBJ, BOOL } kind = NUL;
  double num = 0.0;
  std::string str;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
  const JVal* get(const char* key) const {
    for (const auto& kv : obj)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
};

struct JParser {
  const std::string& s;
  size_t i = 0;
  explicit JParser(const std::string& src) : s(src) {}
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
  }
  bool str(std::string* out) {
    if (i >= s.size() || s[i] != '"') return false;
    ++i;
    out->clear();
    while (i < s.size() && s[i] != '"') {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      out->push_back(s[i++]);
    }
    if (i >= s.size()) return false;
    ++i;
    return true;
  }
  bool value(JVal* v, int depth = 0) {
    if (depth > 32) return false;
    ws();
    if (i >= s.size()) return false;
    const char ch = s[i];
    if (ch == '{') {
      v->kind = JVal::OBJ;
      ++i;
      ws();
      if (i < s.size() && s[i] == '}') { ++i; return true; }
      while (true) {
        ws();
        std::string key;
        if (!str(&key)) return false;
        ws();
        if (i >= s.size() || s[i] != ':') return false;
        ++i;
        JVal child;
        if (!value(&child, depth + 1)) return false;
        v->obj.emplace_back(key, std::move(child));
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; return true; }
        return false;
      }
    }
    if (ch == '[') {
      v->kind = JVal::ARR;
      ++i;
      ws();
      if (i < s.size() && s[i] == ']') { ++i; return true; }
      while (true) {
        JVal child;
        if (!value(&child, depth + 1)) return false;
        v->arr.push_back(std::move(child));
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; return true; }
        return false;
      }
    }
    if (ch == '"') {
      v->kind = JVal::STR;
      return str(&v->str);
    }
    if (s.compare(i, 4, "true") == 0) { v->kind = JVal::BOOL; v->num = 1; i += 4; return true; }
    if (s.compare(i, 5, "false") == 0) { v->kind = JVal::BOOL; i += 5; return true; }
    if (s.compare(i, 4, "null") == 0) { v->kind = JVal::NUL; i += 4; return true; }
    const char* start = s.c_str() + i;
    char* end = nullptr;
    v->num = std::strtod(start, &end);
    if (end == start) return false;
    v->kind = JVal::NUM;
    i += static_cast<size_t>(end - start);
    return true;
  }
};

bool jnums(const JVal* v, double* out, size_t n) {
  if (!v || v->kind != JVal::ARR || v->arr.size() != n) return false;
  for (size_t k = 0; k < n; ++k) {
    if (v->arr[k].kind != JVal::NUM) return false;
    out[k] = v->arr[k].num;
  }
  return true;
}

bool jnum(const JVal* v, double* out) {
  if (!v || v->kind != JVal::NUM) return false;
  *out = v->num;
  return true;
}

std::string kin_library_dir() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&osc_kin_desc_from_json), &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s);
  }
  return ".";
}

}  // namespace

struct osc_kin_model {
  osc_kin_desc desc;
  KinDev host;
  KinDev* dev;
  int device;
};

extern "C" int osc_kin_desc_from_json(const char* robot, const char* json_path,
                                      osc_kin_desc* desc) {
  if (!desc || (!robot && !json_path)) return OSC_ERR_INVALID_ARGUMENT;
  const std::string path = json_path ? std::string(json_path)
                                     : kin_library_dir() + "/../config/" + robot +
                                           "_kinematics.json";
  std::ifstream in(path);
  if (!in) return OSC_ERR_IO;
  std::stringstream ss;
  ss << in.rdbuf();
  const std::string text = ss.str();
  JVal root;
  JParser p(text);
  if (!p.value(&root) || root.kind != JVal::OBJ) {
    std::fprintf(stderr, "osc_kin_desc_from_json: %s: malformed JSON\n", path.c_str());
    return OSC_ERR_IO;
  }
  std::memset(desc, 0, sizeof(*desc));
  const JVal* bodies = root.get("bodies");
  const JVal* sites = root.get("sites");
  if (!bodies || bodies->kind != JVal::ARR || !sites || sites->kind != JVal::ARR ||
      !jnums(root.get("gravity"), desc->gravity, 3))
    return OSC_ERR_IO;
  if (bodies->arr.size() > OSC_KIN_MAX_BODIES || sites->arr.size() > OSC_KIN_MAX_SITES)
    return OSC_ERR_INVALID_ARGUMENT;
  desc->nbody = static_cast<int32_t>(bodies->arr.size());
  desc->nsite = static_cast<int32_t>(sites->arr.size());
  for (int b = 0; b < desc->nbody; ++b) {
    const JVal& B = bodies->arr[b];
    double parent = 0.0;
    const JVal* jt = B.get("joint");
    if (!jnum(B.get("parent"), &parent) || !jt || jt->kind != JVal::STR ||
        !jnums(B.get("pos"), desc->pos[b], 3) || !jnums(B.get("quat"), desc->quat[b], 4) ||
        !jnum(B.get("mass"), &desc->mass[b]) || !jnums(B.get("ipos"), desc->ipos[b], 3) ||
        !jnums(B.get("iquat"), desc->iquat[b], 4) ||
        !jnums(B.get("diaginertia"), desc->inertia[b], 3))
      return OSC_ERR_IO;
    desc->parent[b] = static_cast<int32_t>(parent);
    if (jt->str == "free") desc->jnt_type[b] = OSC_KIN_JOINT_FREE;
    else if (jt->str == "hinge") desc->jnt_type[b] = OSC_KIN_JOINT_HINGE;
    else if (jt->str == "slide") desc->jnt_type[b] = OSC_KIN_JOINT_SLIDE;
    else if (jt->str == "ball") desc->jnt_type[b] = OSC_KIN_JOINT_BALL;
    else if (jt->str == "none") desc->jnt_type[b] = OSC_KIN_JOINT_NONE;
    else return OSC_ERR_IO;
    if (B.get("axis") && !jnums(B.get("axis"), desc->axis[b], 3)) return OSC_ERR_IO;
    if (B.get("jnt_pos") && !jnums(B.get("jnt_pos"), desc->jnt_pos[b], 3)) return OSC_ERR_IO;
    if (B.get("armature") && !jnum(B.get("armature"), &desc->armature[b])) return OSC_ERR_IO;
  }
  for (int s = 0; s < desc->nsite; ++s) {
    const JVal& S = sites->arr[s];
    double body = 0.0;
    if (!jnum(S.get("body"), &body) || !jnums(S.get("pos"), desc->site_pos[s], 3))
      return OSC_ERR_IO;
    desc->site_body[s] = static_cast<int32_t>(body);
    desc->site_jac_body[s] = desc->site_body[s];
    if (const JVal* jb = S.get("jac_body")) {   // optional: Jacobian body != the site's body
      double v = 0.0;
      if (!jnum(jb, &v)) return OSC_ERR_IO;
      desc->site_jac_body[s] = static_cast<int32_t>(v);
      desc->has_jac_body = 1;
    }
  }
  return OSC_OK;
}

extern "C" int osc_kin_model_create(const osc_kin_desc* desc, osc_kin_model** out) {
  if (!desc || !out) return OSC_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  osc_kin_model* m = new (std::nothrow) osc_kin_model;
  if (!m) return OSC_ERR_DEVICE;
  const int rc = build_tables(*desc, &m->host);
  if (rc != OSC_OK) {
    delete m;
    return rc;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    delete m;
    return OSC_ERR_NO_DEVICE;
  }
  m->desc = *desc;
  m->dev = nullptr;
  (void)hipGetDevice(&m->device);
  if (hipMalloc(&m->dev, sizeof(KinDev)) != hipSuccess ||
      hipMemcpy(m->dev, &m->host, sizeof(KinDev), hipMemcpyHostToDevice) != hipSuccess) {
    if (m->dev) (void)hipFree(m->dev);
    delete m;
    return OSC_ERR_DEVICE;
  }
  *out = m;
  return OSC_OK;
}

extern "C" int osc_kin_model_create_from_json(const char* robot, const char* json_path,
                                              osc_kin_model** out) {
  osc_kin_desc d;
  const int rc = osc_kin_desc_from_json(robot, json_path, &d);
  if (rc != OSC_OK) return rc;
  return osc_kin_model_create(&d, out);
}

extern "C" int osc_kin_model_destroy(osc_kin_model* model) {
  if (!model) return OSC_ERR_INVALID_ARGUMENT;
  if (model->dev) (void)hipFree(model->dev);
  delete model;
  return OSC_OK;
}

extern "C" int osc_kin_model_dims(const osc_kin_model* model, int32_t* nq, int32_t* nv,
                                  int32_t* nsite) {
  if (!model) return OSC_ERR_INVALID_ARGUMENT;
  if (nq) *nq = model->host.nq;
  if (nv) *nv = model->host.nv;
  if (nsite) *nsite = model->host.nsite;
  return OSC_OK;
}

extern "C" int osc_batch_kinematics(const osc_kin_model* model, int32_t nenv, const double* qpos,
                                    const double* qvel, double* M, double* C, double* J,
                                    double* b, double* site_xpos, void* stream) {
  if (!model || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!qpos || !qvel || !M || !C || !J || !b) return OSC_ERR_INVALID_ARGUMENT;
  const KinDev& k = model->host;
  const EnvLayout lay(k.nq, k.nv, k.nbody, k.nsite);
  const size_t lds = sizeof(double) * static_cast<size_t>(lay.size) * kEnvPerWave;
  const unsigned nblk = static_cast<unsigned>((nenv + kEnvPerWave - 1) / kEnvPerWave);
  hipLaunchKernelGGL(osc_kinematics_kernel, dim3(nblk), dim3(kWave), lds,
                     static_cast<hipStream_t>(stream), model->dev, nenv, qpos, qvel, M, C, J, b,
                     site_xpos);
  return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}

extern "C" int osc_state_to_qpos(int32_t nenv, int32_t nu, const double* body_rotation,
                                 const double* linear_body_velocity,
                                 const double* angular_body_velocity,
                                 const double* motor_position, const double* motor_velocity,
                                 double* qpos, double* qvel, void* stream) {
  if (nenv < 0 || nu < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if (!body_rotation || !linear_body_velocity || !angular_body_velocity || !qpos || !qvel ||
      (nu > 0 && (!motor_position || !motor_velocity)))
    return OSC_ERR_INVALID_ARGUMENT;
  const long long total = static_cast<long long>(nenv) * (13 + 2 * nu);
  const unsigned nblk = static_cast<unsigned>(std::min<long long>((total + kPackBlock - 1) /
                                                                  kPackBlock, 4096));
  hipLaunchKernelGGL(state_to_qpos_kernel, dim3(nblk), dim3(kPackBlock), 0,
                     static_cast<hipStream_t>(stream), nenv, nu, body_rotation,
                     linear_body_velocity, angular_body_velocity, motor_position, motor_velocity,
                     qpos, qvel);
  return hipGetLastError() == hipSuccess ? OSC_OK : OSC_ERR_DEVICE;
}

namespace {

size_t align256(size_t n) { return (n + 255) & ~static_cast<size_t>(255); }

struct QposWorkspace {   // [M | C | J | b | reduced-QP workspace], each section 256-B aligned
  size_t m, c, j, b, ws, ws_bytes, total;
  QposWorkspace(const osc_model* model, const KinDev& k, int32_t nenv) {
    const size_t n = static_cast<size_t>(nenv);
    m = 0;
    c = m + align256(sizeof(double) * n * k.nv * k.nv);
    j = c + align256(sizeof(double) * n * k.nv);
    b = j + align256(sizeof(double) * n * 6 * k.nsite * k.nv);
    ws = b + align256(sizeof(double) * n * 6 * k.nsite);
    ws_bytes = 0;
    osc_workspace_bytes(model, nenv, &ws_bytes);
    total = ws + align256(ws_bytes);
  }
};

int check_pair(const osc_model* model, const osc_kin_model* kin) {
  if (!model || !kin) return OSC_ERR_INVALID_ARGUMENT;
  osc_model_desc d;
  if (osc_model_get_desc(model, &d) != OSC_OK) return OSC_ERR_INVALID_ARGUMENT;
  if (d.nv != kin->host.nv || d.ns != kin->host.nsite) return OSC_ERR_INVALID_ARGUMENT;
  return OSC_OK;
}

}  // namespace

extern "C" int osc_qpos_workspace_bytes(const osc_model* model, const osc_kin_model* kin,
                                        int32_t nenv, size_t* bytes) {
  if (!bytes || nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  const int rc = check_pair(model, kin);
  if (rc != OSC_OK) return rc;
  *bytes = QposWorkspace(model, kin->host, nenv).total;
  return OSC_OK;
}

namespace {

int solve_qpos(const osc_model* model, const osc_kin_model* kin, int32_t nenv, const double* qpos,
               const double* qvel, const double* T, const double* contact_mask, double* tau,
               double* x, int32_t* status, int32_t* iters, double* warm_state,
               size_t warm_state_bytes, void* workspace,
               size_t workspace_bytes, void* stream) {
  int rc = check_pair(model, kin);
  if (rc != OSC_OK) return rc;
  if (nenv < 0) return OSC_ERR_INVALID_ARGUMENT;
  if (nenv == 0) return OSC_OK;
  if ((reinterpret_cast<uintptr_t>(workspace) & 15u) != 0) return OSC_ERR_INVALID_ARGUMENT;
  const QposWorkspace L(model, kin->host, nenv);
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* base = static_cast<char*>(workspace);
  bool owned = false;
  if (base == nullptr) {
    if (hipMallocAsync(reinterpret_cast<void**>(&base), L.total, s) != hipSuccess)
      return OSC_ERR_DEVICE;
    owned = true;
  } else if (workspace_bytes < L.total) {
    return OSC_ERR_INVALID_ARGUMENT;
  }
  // The tick as two kernels: osc_batch_kinematics (four envs per wave, one round of waves at
  // 4,096 envs) then osc_batch_solve.  (-DOSC_FUSED_TICK builds the fused tick instead -- the
  // kinematics in the assembly kernel's prologue, osc_setup.hpp setup_env<D, true>, bitwise the
  // same results -- measured slower at every size: Go2 4,096 0.1947 vs 0.1882 ms, 65,536 2.177
  // vs 2.053 ms, WaLTER 4,096 0.286 vs 0.262 ms (profiles/r05/tick_ab_fused.jsonl): one env per
  // wave pays the tree's level-by-level latency once per round of assembly waves, where the
  // separate kernel pays it once for four envs.)
#ifdef OSC_FUSED_TICK
  (void)L.m;
  if (!qpos || !qvel) rc = OSC_ERR_INVALID_ARGUMENT;
  const osc::QposArgs q{kin->dev, kin->host.nq, kin->host.nbody, qpos, qvel};
  if (rc == OSC_OK)
    rc = osc::solve_qpos_fused(model, q, nenv, T, contact_mask, tau, x, status, iters, warm_state,
                               warm_state_bytes, base + L.ws, L.ws_bytes, stream);
#else
  double* M = reinterpret_cast<double*>(base + L.m);
  double* C = reinterpret_cast<double*>(base + L.c);
  double* J = reinterpret_cast<double*>(base + L.j);
  double* b = reinterpret_cast<double*>(base + L.b);
  rc = osc_batch_kinematics(kin, nenv, qpos, qvel, M, C, J, b, nullptr, stream);
  if (rc == OSC_OK)
    rc = warm_state ? osc_batch_solve_warm(model, nenv, M, C, J, b, T, contact_mask, tau, x,
                                           status, iters, warm_state, warm_state_bytes,
                                           base + L.ws, L.ws_bytes, stream)
                    : osc_batch_solve(model, nenv, M, C, J, b, T, contact_mask, tau, x, status,
                                      iters, base + L.ws, L.ws_bytes, stream);
#endif
  if (owned) (void)hipFreeAsync(base, s);
  return rc;
}

}  // namespace

extern "C" int osc_batch_solve_qpos(const osc_model* model, const osc_kin_model* kin,
                                    int32_t nenv, const double* qpos, const double* qvel,
                                    const double* T, const double* contact_mask, double* tau,
                                    double* x, int32_t* status, int32_t* iters, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  return solve_qpos(model, kin, nenv, qpos, qvel, T, contact_mask, tau, x, status, iters, nullptr,
                    0, workspace, workspace_bytes, stream);
}

extern "C" int osc_batch_solve_qpos_warm(const osc_model* model, const osc_kin_model* kin,
                                         int32_t nenv, const double* qpos, const double* qvel,
                                         const double* T, const double* contact_mask, double* tau,
                                         double* x, int32_t* status, int32_t* iters,
                                         double* warm_state, size_t warm_state_bytes,
                                         void* workspace, size_t workspace_bytes, void* stream) {
  if (!warm_state) return OSC_ERR_INVALID_ARGUMENT;
  return solve_qpos(model, kin, nenv, qpos, qvel, T, contact_mask, tau, x, status, iters,
                    warm_state, warm_state_bytes, workspace, workspace_bytes, stream);
}
