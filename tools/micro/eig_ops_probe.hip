// Cost of the operations on eigmin_split's per-column path, one workgroup of 576 threads (9
// waves: 2-3 per SIMD, as the kernel runs), each op repeated R times between two s_memtime
// stamps (cycles per repetition, wave 0 / wave 4 / all waves doing it):
//   fma32dpp  : 32 v_fmac_f64_dpp row_newbcast into 4 chains (the matvec of one column)
//   fma64dpp  : 64 v_fmac_f64_dpp into 32 independent accumulators (the rank-2 update)
//   fma64     : 64 plain v_fmac_f64 (the same without DPP)
//   xsum      : xsum32(xsum16(x)) (cross-class sum of p)
//   row16     : row16_sum (4 DPP steps: v^T p partials, reflector norm)
//   wavesum   : row16 + xsum (a full 64-lane sum)
//   ldsbar    : LDS write, barrier, LDS read (one round trip through a barrier)
//   bar       : barrier alone
//   rsqrcp    : Newton-refined rsq then rcp chain (the reflector's scalars)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form eig_ops_probe.hip -o eig_ops_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../clustered-low-rank-sdp-solver_amd/csrc/kernels_dense.h"
using namespace clrsdp;

constexpr int R = 200;

template <int OP>
__global__ __launch_bounds__(576) void probe(double* out, unsigned long long* cyc) {
  __shared__ double buf[2][576];
  const int tid = threadIdx.x, w = tid >> 6;
  double acc[32];
#pragma unroll
  for (int q = 0; q < 32; ++q) acc[q] = q * 1e-3 + tid;
  double x = tid * 1e-7, m = 1.0 + tid * 1e-9;
  buf[0][tid] = x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < R; ++it) {
    if constexpr (OP == 0) {
      double pa[4] = {0, 0, 0, 0};
      static_for<0, 16>([&](auto S) {
        constexpr int s = decltype(S)::value;
        fmac_bcast<s, (s & 3) == 0>(pa[2 * (s & 1)], x, acc[2 * s]);
        fmac_bcast<s, false>(pa[2 * (s & 1) + 1], x, acc[2 * s + 1]);
      });
      x = (pa[0] + pa[1]) + (pa[2] + pa[3]);
    } else if constexpr (OP == 1) {
      static_for<0, 16>([&](auto S) {
        constexpr int s = decltype(S)::value;
        fmac_bcast<s, (s & 3) == 0>(acc[2 * s], x, m);
        fmac_bcast<s, false>(acc[2 * s + 1], x, m);
      });
      static_for<0, 16>([&](auto S) {
        constexpr int s = decltype(S)::value;
        fmac_bcast<s, false>(acc[2 * s], m, x);
        fmac_bcast<s, false>(acc[2 * s + 1], m, x);
      });
    } else if constexpr (OP == 2) {
#pragma unroll
      for (int q = 0; q < 32; ++q) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(acc[q]) : "v"(x), "v"(m));
#pragma unroll
      for (int q = 0; q < 32; ++q) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(acc[q]) : "v"(m), "v"(x));
    } else if constexpr (OP == 3) {
      x = xsum32(xsum16(x)) * 0.25;
    } else if constexpr (OP == 4) {
      x = row16_sum(x) * 0.0625;
    } else if constexpr (OP == 5) {
      x = xsum32(xsum16(row16_sum(x))) * (1.0 / 64);
    } else if constexpr (OP == 6) {
      buf[it & 1][tid] = x;
      __syncthreads();
      x = buf[it & 1][(tid + 64) % 576] * 0.5 + 1.0;
    } else if constexpr (OP == 7) {
      __syncthreads();
      x = x * m;
    } else if constexpr (OP == 8) {
      const double ss = x * x + 1.0;
      double rs = __builtin_amdgcn_rsq(ss);
      rs = rs * fma(-0.5 * ss, rs * rs, 1.5);
      double nrm = ss * rs;
      nrm = fma(fma(-nrm, nrm, ss), 0.5 * rs, nrm);
      const double q = fma(nrm, nrm, 1.0);
      double rc = __builtin_amdgcn_rcp(q);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      rc = fma(fma(-q, rc, 1.0), rc, rc);
      x = rc * 1e-3;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = x;
#pragma unroll
  for (int q = 0; q < 32; ++q) s += acc[q];
  out[blockIdx.x * 576 + tid] = s;
  if ((tid & 63) == 0) cyc[blockIdx.x * 9 + w] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 128 * 576 * 8);
  (void)hipMalloc(&cyc, 128 * 9 * 8);
  const char* names[] = {"fma32dpp (4 chains)", "fma64dpp (32 acc)", "fma64 plain", "xsum16+32",
                         "row16_sum", "wave sum (64)", "lds write-bar-read", "barrier", "rsq+rcp chain"};
  for (int op = 0; op < 9; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (op) {
        case 0: probe<0><<<128, 576>>>(out, cyc); break;
        case 1: probe<1><<<128, 576>>>(out, cyc); break;
        case 2: probe<2><<<128, 576>>>(out, cyc); break;
        case 3: probe<3><<<128, 576>>>(out, cyc); break;
        case 4: probe<4><<<128, 576>>>(out, cyc); break;
        case 5: probe<5><<<128, 576>>>(out, cyc); break;
        case 6: probe<6><<<128, 576>>>(out, cyc); break;
        case 7: probe<7><<<128, 576>>>(out, cyc); break;
        case 8: probe<8><<<128, 576>>>(out, cyc); break;
      }
      (void)hipDeviceSynchronize();
    }
    unsigned long long c[9];
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-22s cycles per repetition: wave0 %7.1f  wave4 %7.1f  wave8 %7.1f\n", names[op],
           c[0] / (double)R, c[4] / (double)R, c[8] / (double)R);
  }
  return 0;
}
