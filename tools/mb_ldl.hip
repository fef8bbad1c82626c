// Microbenchmark (diagnostic, not product): throughput of a register-resident LDL^T of an
// N x N SPD matrix under different wavefront mappings.
//   V1: 1 env / wave, lane j holds column j, pivot column broadcast with v_readlane
//   V2: 2 env / wave (32-lane groups), broadcast with ds_swizzle (bitmask mode, or_mask = k)
//   V3: 2 env / wave, broadcast with two v_readlane (lane k and 32+k) + per-half select
//   V4: 4 env / wave (16-lane groups), 2 columns per lane, ds_swizzle broadcast
// Each thread factorises its column(s) REPS times; time / (REPS * envs) = cost per env-LDL^T.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <type_traits>
#include <vector>

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ int opaque(int x) { asm volatile("" : "+v"(x)); return x; }

__device__ __forceinline__ double rl(double v, int k) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}
template <int PAT>
__device__ __forceinline__ double swz(double v) {
  int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), PAT);
  int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), PAT);
  return __hiloint2double(hi, lo);
}
// bitmask mode: lane' = ((lane & and) | or) ^ xor inside each group of 32
template <int K, int GROUP>
__device__ __forceinline__ double gbcast(double v) {
  constexpr int and_mask = (GROUP == 32) ? 0 : (32 - GROUP);   // keep the group bits
  return swz<(0 << 10) | (K << 5) | and_mask>(v);
}

template <int N>
__device__ void init_col(double (&c)[N], int j, int seed) {
#pragma unroll
  for (int i = 0; i < N; ++i) c[i] = (i == j ? 2.0 * N : 0.0) + 1.0 / (1 + ((i + j + seed) % 7));
}

template <int N, int REPS>
__global__ __launch_bounds__(64) void v1(double* out) {
  const int lane = threadIdx.x;
  double c[N];
  double acc = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    init_col<N>(c, lane, rep);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const double dk = rl(c[k], k);
      const double inv = 1.0 / dk;
      const int ln = opaque(lane);
      const double t = (ln > k && ln < N) ? c[k] * inv : 0.0;
#pragma unroll
      for (int i = k + 1; i < N; ++i) c[i] = fma(-rl(c[i], k), t, c[i]);
    }
    acc += c[N - 1];
  }
  out[blockIdx.x * 64 + lane] = acc;
}

template <int N, int REPS>
__global__ __launch_bounds__(64) void v2(double* out) {
  const int lane = threadIdx.x, l = lane & 31;
  double c[N];
  double acc = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    init_col<N>(c, l, rep);
    static_for<0, N>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const double dk = gbcast<k, 32>(c[k]);
      const double inv = 1.0 / dk;
      const int ln = opaque(l);
      const double t = (ln > k && ln < N) ? c[k] * inv : 0.0;
      static_for<k + 1, N>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        c[i] = fma(-gbcast<k, 32>(c[i]), t, c[i]);
      });
    });
    acc += c[N - 1];
  }
  out[blockIdx.x * 64 + lane] = acc;
}

// 2 env / wave with ds_bpermute (runtime lane address) instead of ds_swizzle
__device__ __forceinline__ double bperm(double v, int addr) {
  int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
template <int N, int REPS>
__global__ __launch_bounds__(64) void v2b(double* out) {
  const int lane = threadIdx.x, l = lane & 31;
  const int base = (lane & 32) << 2;
  double c[N];
  double acc = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    init_col<N>(c, l, rep);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const int addr = base + 4 * k;
      const double dk = bperm(c[k], addr);
      const double inv = 1.0 / dk;
      const int ln = opaque(l);
      const double t = (ln > k && ln < N) ? c[k] * inv : 0.0;
#pragma unroll
      for (int i = k + 1; i < N; ++i) c[i] = fma(-bperm(c[i], addr), t, c[i]);
    }
    acc += c[N - 1];
  }
  out[blockIdx.x * 64 + lane] = acc;
}

template <int N, int REPS>
__global__ __launch_bounds__(64) void v3(double* out) {
  const int lane = threadIdx.x, l = lane & 31;
  const bool hi = lane >= 32;
  double c[N];
  double acc = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    init_col<N>(c, l, rep);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const double d0 = rl(c[k], k), d1 = rl(c[k], k + 32);
      const double dk = hi ? d1 : d0;
      const double inv = 1.0 / dk;
      const int ln = opaque(l);
      const double t = (ln > k && ln < N) ? c[k] * inv : 0.0;
#pragma unroll
      for (int i = k + 1; i < N; ++i) {
        const double a0 = rl(c[i], k), a1 = rl(c[i], k + 32);
        c[i] = fma(-(hi ? a1 : a0), t, c[i]);
      }
    }
    acc += c[N - 1];
  }
  out[blockIdx.x * 64 + lane] = acc;
}

// 4 envs per wave: 16-lane groups, lane l holds columns l and l+16 (N <= 32)
template <int N, int REPS>
__global__ __launch_bounds__(64) void v4(double* out) {
  const int lane = threadIdx.x, l = lane & 15;
  double c0[N], c1[N];
  double acc = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    init_col<N>(c0, l, rep);
    init_col<N>(c1, l + 16, rep);
    static_for<0, N>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      double dk;
      if constexpr (k < 16) dk = gbcast<k % 16, 16>(c0[k]); else dk = gbcast<k % 16, 16>(c1[k]);
      const double inv = 1.0 / dk;
      const int ln = opaque(l);
      const double t0 = (ln > k && ln < N) ? c0[k] * inv : 0.0;
      const double t1 = (ln + 16 > k && ln + 16 < N) ? c1[k] * inv : 0.0;
      static_for<k + 1, N>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        double b;
        if constexpr (k < 16) b = gbcast<k % 16, 16>(c0[i]); else b = gbcast<k % 16, 16>(c1[i]);
        c0[i] = fma(-b, t0, c0[i]);
        c1[i] = fma(-b, t1, c1[i]);
      });
    });
    acc += c0[N - 1] + c1[N - 1];
  }
  out[blockIdx.x * 64 + lane] = acc;
}


// V5: 4 envs / wave, one 16-lane DPP row per env, 2 columns per lane, pivot column broadcast
// with v_mov_b64_dpp row_newbcast (VALU, no LDS pipe), reciprocal by rcp + 2 Newton steps.
template <int K>
__device__ __forceinline__ double rowb(double v) {
  long long x = __double_as_longlong(v);
  return __longlong_as_double(__builtin_amdgcn_mov_dpp(x, 0x150 + K, 0xf, 0xf, false));
}
__device__ __forceinline__ double recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}
template <int N, int REPS>
__global__ __launch_bounds__(64) void v5(double* out) {
  const int lane = threadIdx.x, l = lane & 15;
  double c0[N], c1[N];
  double acc = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    init_col<N>(c0, l, rep);
    init_col<N>(c1, l + 16, rep);
    static_for<0, N>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      double dk;
      if constexpr (k < 16) dk = rowb<k % 16>(c0[k]); else dk = rowb<k % 16>(c1[k]);
      const double inv = recip(dk);
      const int ln = opaque(l);
      const double t0 = (ln > k && ln < N) ? -c0[k] * inv : 0.0;
      const double t1 = (ln + 16 > k && ln + 16 < N) ? -c1[k] * inv : 0.0;
      static_for<k + 1, N>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        double b;
        if constexpr (k < 16) b = rowb<k % 16>(c0[i]); else b = rowb<k % 16>(c1[i]);
        c0[i] = fma(b, t0, c0[i]);
        if constexpr (N > 16) c1[i] = fma(b, t1, c1[i]);
      });
    });
    acc += c0[N - 1] + c1[N - 1];
  }
  out[blockIdx.x * 64 + lane] = acc;
}

template <class F>
float time_it(F kern, int blocks, double* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

template <int N>
void run() {
  constexpr int REPS = 64;
  const int blocks = 256 * 32;   // 32 waves per CU worth of blocks
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * 64);
  float t1 = time_it(v1<N, REPS>, blocks, out);
  float t2 = time_it(v2<N, REPS>, blocks, out);
  float t3 = time_it(v3<N, REPS>, blocks, out);
  float t4 = time_it(v4<N, REPS>, blocks, out);
  float t2b = time_it(v2b<N, REPS>, blocks, out);
  float t5 = time_it(v5<N, REPS>, blocks, out);
  auto per = [&](float ms, int envs_per_wave) { return ms * 1e6 / (double(blocks) * envs_per_wave * REPS); };
  printf("{\"N\": %d, \"ns_per_env_ldl\": {\"v1_readlane_1env\": %.3f, \"v2_swizzle_2env\": %.3f, "
         "\"v3_readlane_2env\": %.3f, \"v4_swizzle_4env\": %.3f, \"v2b_bpermute_2env\": %.3f, \"v5_dpp_4env\": %.3f}}\n",
         N, per(t1, 1), per(t2, 2), per(t3, 2), per(t4, 4), per(t2b, 2), per(t5, 4));
  hipFree(out);
}

int main() {
  run<24>();
  run<32>();
  return 0;
}
