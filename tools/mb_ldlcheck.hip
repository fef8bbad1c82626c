// Correctness harness for the IPM kernel's row-group LDL^T + solve (device functions included
// from the product source).  4 row groups x N=24 SPD systems; max error vs host solve.
#include "../operational-space-control_amd/csrc/osc_batch.hip"
#include <cmath>
#include <cstdio>
#include <vector>

template <int N>
__global__ void k_check(const double* K, const double* r, double* x, double* F) {
  const int lane = threadIdx.x, grp = lane / kRow, l = lane % kRow;
  __shared__ double sdg[4][N];
  __shared__ double sdinv[4][2 * kRow];
  const double* Kg = K + grp * N * N;
  double c0[N], c1[N];
  const int j1 = l + kRow < N ? l + kRow : N - 1;
  for (int i = 0; i < N; ++i) {
    c0[i] = Kg[i * N + l];
    c1[i] = Kg[i * N + j1];
  }
  sdg[grp][l] = Kg[l * N + l];
  if (l + kRow < N) sdg[grp][l + kRow] = Kg[j1 * N + j1];
  __syncthreads();
  double d0, d1;
  ldl_rows<N>(c0, c1, sdinv[grp], l, d0, d1, 1e-13 * Kg[l * N + l], 1e-13 * Kg[j1 * N + j1]);  // d0/d1 = 1/D
  for (int i = 0; i < N; ++i) {
    F[grp * N * N + i * N + l] = c0[i];
    if (l + kRow < N) F[grp * N * N + i * N + l + kRow] = c1[i];
  }
  F[4 * N * N + grp * N + l] = d0;
  if (l + kRow < N) F[4 * N * N + grp * N + l + kRow] = d1;
  double a0 = r[grp * N + l], a1 = r[grp * N + j1];
  ldl_solve_rows<N>(c0, c1, d0, d1, a0, a1, l);
  x[grp * N + l] = a0;
  if (l + kRow < N) x[grp * N + l + kRow] = a1;
}

int main() {
  constexpr int N = 24;
  std::vector<double> K(4 * N * N), r(4 * N), x(4 * N);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
  for (int g = 0; g < 4; ++g) {
    std::vector<double> A(N * N);
    for (auto& v : A) v = rnd();
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        double acc = (i == j) ? N : 0.0;
        for (int k = 0; k < N; ++k) acc += A[i * N + k] * A[j * N + k];
        K[g * N * N + i * N + j] = acc;
      }
    for (int i = 0; i < N; ++i) r[g * N + i] = rnd();
  }
  double *dK, *dr, *dx, *dF;
  std::vector<double> F(4 * N * N + 4 * N);
  (void)hipMalloc(&dF, F.size() * 8);
  (void)hipMalloc(&dK, K.size() * 8); (void)hipMalloc(&dr, r.size() * 8); (void)hipMalloc(&dx, x.size() * 8);
  (void)hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dr, r.data(), r.size() * 8, hipMemcpyHostToDevice);
  k_check<N><<<1, 64>>>(dK, dr, dx, dF);
  (void)hipMemcpy(F.data(), dF, F.size() * 8, hipMemcpyDeviceToHost);
  {  // host LDL^T of group 0
    std::vector<double> A(K.begin(), K.begin() + N * N), L(N * N, 0.0), Dg(N);
    for (int k = 0; k < N; ++k) {
      Dg[k] = A[k * N + k];
      for (int i = k + 1; i < N; ++i) L[i * N + k] = A[i * N + k] / Dg[k];
      for (int i = k + 1; i < N; ++i)
        for (int j = k + 1; j < N; ++j) A[i * N + j] -= L[i * N + k] * Dg[k] * L[j * N + k];
    }
    double ecol = 0, erow = 0, ediag = 0, edinv = 0; int bi = -1, bj = -1;
    for (int j = 0; j < N; ++j) {
      for (int i = 0; i < N; ++i) {
        double f = F[i * N + j];
        // ldl_rows' output: row k of every column pre-scaled by -1/D_k (the diagonal -> -1)
        if (i > j) { double e = fabs(f + L[i * N + j] * Dg[j] / Dg[i]); if (e > ecol) { ecol = e; bi = i; bj = j; } }
        if (i < j) erow = fmax(erow, fabs(f + L[j * N + i]));
        if (i == j) ediag = fmax(ediag, fabs(f + 1.0));
      }
      edinv = fmax(edinv, fabs(F[4 * N * N + j] * Dg[j] - 1.0));
    }
    printf("factor errors: col %g (at %d,%d) row %g diag %g dinv %g\n", ecol, bi, bj, erow, ediag, edinv);
  }
  (void)hipMemcpy(x.data(), dx, x.size() * 8, hipMemcpyDeviceToHost);
  double worst = 0;
  for (int g = 0; g < 4; ++g)
    for (int i = 0; i < N; ++i) {
      double acc = -r[g * N + i];
      for (int j = 0; j < N; ++j) acc += K[g * N * N + i * N + j] * x[g * N + j];
      worst = fmax(worst, fabs(acc));
      if (g == 0 && i < 24) printf("%d x=%g res=%g\n", i, x[i], acc);
    }
  printf("max residual %g -> %s\n", worst, worst < 1e-10 ? "OK" : "BAD");
  return worst < 1e-10 ? 0 : 1;
}
