// Microbenchmark (diagnostic, not product): the IPM's Newton-matrix LDL^T at the occupancy of a
// resident batch, in the product's layout and in the two-env, 32-lane layout VERDICT r2 #4 asks
// about.  Both factorise 24 x 24 SPD matrices (Go2's NY) REPS times per wave; the grid is sized
// so that the SAME number of envs is in flight (e.g. 4,096: 1,024 vs 2,048 waves), every wave
// resident at once.
//   A (product): 4 envs / wave, one 16-lane DPP row each, lane l holds columns l and l+16
//     (ldl_rows of csrc/osc_batch.hip, included below: the factor the kernel runs), one wave
//     per SIMD at 4,096 envs.
//   B: 2 envs / wave, 32 lanes each: both 16-lane rows of an env hold columns l and l+16, row r
//     the entries i = r (mod 2) -- so a pivot column's entries are DPP-broadcast inside each row
//     as in A, and half the trailing FMAs per lane; the pivot and the multipliers -L[j][k] cross
//     between the two rows (__shfl_xor 16) once per step.  Two waves per SIMD at 4,096 envs.
// Each variant's factor is checked against a host LDL^T of the same matrix.  Dynamic LDS pads
// pin the residency the product has: A <= 4 workgroups per CU (one wave per SIMD, as the
// kernel's padded LDS request does), B <= 8 (two per SIMD).
#include "../operational-space-control_amd/csrc/osc_batch.hip"
#include <cmath>
#include <cstdio>
#include <vector>

constexpr int N = 24, REPS = 20, M2 = N / 2;

__device__ __forceinline__ double kval(int i, int j, int env) {   // SPD, diagonally dominant
  const double off = 1.0 / (1.0 + ((i * 7 + j * 7 + (i == j ? 0 : i * j) + env) % 11));
  return i == j ? 2.0 * N : off;
}

__global__ __launch_bounds__(64, 1) void k_a(double* out, int nenv) {
  __shared__ double sdinv[4][2 * kRow];
  const int lane = threadIdx.x, grp = lane / kRow, l = lane % kRow;
  const int env = blockIdx.x * 4 + grp;
  const int j1 = l + kRow < N ? l + kRow : N - 1;
  double k0[N], k1[N];
  for (int i = 0; i < N; ++i) {
    k0[i] = kval(i, l, env);
    k1[i] = kval(i, j1, env);
  }
  double acc = 0.0;
  for (int rep = 0; rep < REPS; ++rep) {
    double c0[N], c1[N];
    for (int i = 0; i < N; ++i) {
      c0[i] = k0[i] + 1e-3 * rep;
      c1[i] = k1[i] + 1e-3 * rep;
    }
    double d0, d1;
    ldl_rows<N>(c0, c1, sdinv[grp], l, d0, d1, 1e-13 * k0[l], 1e-13 * k1[j1]);
    acc += d0 + d1;
    if (rep == REPS - 1 && env < nenv)
      for (int i = 0; i < N; ++i) {
        out[(size_t)env * N * N + i * N + l] = c0[i];
        if (l + kRow < N) out[(size_t)env * N * N + i * N + l + kRow] = c1[i];
      }
  }
  if (acc == 12345.678) out[0] = acc;   // keep the loop
}

__device__ __forceinline__ double xrow(double v) {   // the other row of the env's row pair
  return __shfl_xor(v, 16);
}

__global__ __launch_bounds__(64, 2) void k_b(double* out, int nenv) {
  __shared__ double sdinv[2][2][2 * kRow];
  const int lane = threadIdx.x, e2 = lane >> 5, r = (lane >> 4) & 1, l = lane & 15;
  const int env = blockIdx.x * 2 + e2;
  const int j1 = l + kRow < N ? l + kRow : N - 1;
  double k0[M2], k1[M2];                      // entries i = 2m + r of columns l, j1
  for (int m = 0; m < M2; ++m) {
    k0[m] = kval(2 * m + r, l, env);
    k1[m] = kval(2 * m + r, j1, env);
  }
  double acc = 0.0;
  for (int rep = 0; rep < REPS; ++rep) {
    double e0[M2], e1[M2];
    for (int m = 0; m < M2; ++m) {
      e0[m] = k0[m] + 1e-3 * rep;
      e1[m] = k1[m] + 1e-3 * rep;
    }
    static_for<0, N>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int ro = k & 1, mk = k >> 1, s = k / kRow, kl = k % kRow;
      // rows 0 / 2 hold the even entries, rows 1 / 3 the odd ones (compile-time lane masks)
      constexpr unsigned long long kOwner = ro == 0 ? 0x0000FFFF0000FFFFull : 0xFFFF0000FFFF0000ull;
      constexpr unsigned long long kRow1 = 0xFFFF0000FFFF0000ull;
      // pivot D_k: lane kl of the owner row, then to the other row
      const double own = (s == 0) ? e0[mk] : e1[mk];
      const double dr = bcast_guarded<kl>(own);
      const double dk = select_lanes<kOwner>(dr, xrow(dr));
      const double inv = recip1(dk);
      if (r == ro) sdinv[e2][r][k] = inv;
      // multipliers -L[j][k] = -c_j[k] / D_k from the owner row (its entry mk is row k)
      const double t0o = -e0[mk] * inv, t1o = -e1[mk] * inv;
      double t0 = select_lanes<kOwner>(t0o, xrow(t0o));
      double t1 = select_lanes<kOwner>(t1o, xrow(t1o));
      t0 = keep_lanes<rows_mask(lanes_from(k + 1, 15))>(t0);   // slot-0 columns still to go
      constexpr unsigned kT1 = (k < kRow) ? lanes_from(0, N - 1 - kRow)
                                          : lanes_from(k + 1 - kRow, N - 1 - kRow);
      t1 = keep_lanes<rows_mask(kT1)>(t1);
      // at m == mk only row 1 of an even k has an entry (2 mk + 1) below the pivot
      const double tm0 = keep_lanes<kRow1>(t0), tm1 = keep_lanes<kRow1>(t1);
      static_for<mk, M2>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        if constexpr (m == mk && ro == 1) return;
        const double u0 = (m == mk) ? tm0 : t0;
        const double u1 = (m == mk) ? tm1 : t1;
        if constexpr (s == 0) {
          fmac_bcast<kl>(e1[m], e0[m], u1);
          fmac_bcast_self<kl>(e0[m], u0);
        } else {
          fmac_bcast_self<kl>(e1[m], u1);
        }
      });
    });
    acc += e0[0] + e1[0];
    if (rep == REPS - 1 && env < nenv)
      for (int m = 0; m < M2; ++m) {
        out[(size_t)env * N * N + (2 * m + r) * N + l] = e0[m];
        if (l + kRow < N) out[(size_t)env * N * N + (2 * m + r) * N + l + kRow] = e1[m];
      }
  }
  if (acc == 12345.678) out[0] = acc;
}

// host: the expected column j entries below the diagonal after the right-looking elimination,
// L[i][j] D_j (both kernels leave them in column j's registers i > j)
static double check(const std::vector<double>& F, int env, bool prescaled_rows) {
  std::vector<double> A(N * N), L(N * N, 0.0), D(N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      const double off = 1.0 / (1.0 + ((i * 7 + j * 7 + (i == j ? 0 : i * j) + env) % 11));
      A[i * N + j] = (i == j ? 2.0 * N : off) + 1e-3 * (REPS - 1);
    }
  for (int k = 0; k < N; ++k) {
    D[k] = A[k * N + k];
    for (int i = k + 1; i < N; ++i) L[i * N + k] = A[i * N + k] / D[k];
    for (int i = k + 1; i < N; ++i)
      for (int j = k + 1; j < N; ++j) A[i * N + j] -= L[i * N + k] * D[k] * L[j * N + k];
  }
  double e = 0.0;
  for (int j = 0; j < N; ++j)
    for (int i = j + 1; i < N; ++i) {
      const double want = prescaled_rows ? -L[i * N + j] * D[j] / D[i] : L[i * N + j] * D[j];
      e = fmax(e, fabs(F[(size_t)env * N * N + i * N + j] - want));
    }
  return e;
}

int main() {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int nenv : {4096, 8192, 16384}) {
    double* d;
    (void)hipMalloc(&d, sizeof(double) * (size_t)nenv * N * N);
    float ta = 1e9f, tb = 1e9f;
    for (int t = 0; t < 5; ++t) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k_a, dim3(nenv / 4), dim3(64), 33 * 1024, 0, d, nenv);   // <= 4 WG / CU
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (t) ta = fminf(ta, ms);
    }
    std::vector<double> F((size_t)nenv * N * N);
    (void)hipMemcpy(F.data(), d, F.size() * 8, hipMemcpyDeviceToHost);
    const double ea = fmax(check(F, 0, true), check(F, nenv - 1, true));
    for (int t = 0; t < 5; ++t) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k_b, dim3(nenv / 2), dim3(64), 18 * 1024, 0, d, nenv);   // <= 8 WG / CU
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (t) tb = fminf(tb, ms);
    }
    (void)hipMemcpy(F.data(), d, F.size() * 8, hipMemcpyDeviceToHost);
    const double eb = fmax(check(F, 1, false), check(F, nenv - 1, false));
    printf("{\"nenv\": %d, \"reps\": %d, \"A_4env_ms\": %.4f, \"B_2env_ms\": %.4f, \"B_over_A\": %.3f, "
           "\"A_us_per_ldl\": %.3f, \"B_us_per_ldl\": %.3f, \"A_err\": %.2e, \"B_err\": %.2e}\n",
           nenv, REPS, ta, tb, tb / ta, ta * 1e3 / REPS, tb * 1e3 / REPS, ea, eb);
    (void)hipFree(d);
  }
  return 0;
}
