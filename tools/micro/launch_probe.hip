// Fixed cost of a launch on MI355X as a function of the grid shape: empty kernels, back to back
// (stream order) and alone (events around one launch).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)
template <int NT> __global__ __launch_bounds__(NT) void empty_k(double* p) { if (threadIdx.x == 9999) p[0] = 1; }
template <int NT> __global__ __launch_bounds__(NT) void touch_k(double* p) {  // one store per thread
  p[blockIdx.x * NT + threadIdx.x] = 1.0;
}
int main() {
  double* buf; CK(hipMalloc(&buf, 64 << 20));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto run = [&](const char* nm, auto go) {
    go(); CK(hipStreamSynchronize(s));
    float tot = 0; const int R = 50;
    for (int r = 0; r < R; ++r) {
      CK(hipEventRecord(e0, s)); go(); CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); tot += ms;
    }
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 200; ++r) go();
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s alone %6.2f us   back-to-back %6.2f us\n", nm, tot * 1e3f / R, ms * 1e3f / 200);
  };
  run("empty    1 x 64", [&] { empty_k<64><<<1, 64, 0, s>>>(buf); });
  run("empty  256 x 64", [&] { empty_k<64><<<256, 64, 0, s>>>(buf); });
  run("empty  256 x 256", [&] { empty_k<256><<<256, 256, 0, s>>>(buf); });
  run("empty  256 x 512", [&] { empty_k<512><<<256, 512, 0, s>>>(buf); });
  run("empty  256 x 1024", [&] { empty_k<1024><<<256, 1024, 0, s>>>(buf); });
  run("empty 1024 x 256", [&] { empty_k<256><<<1024, 256, 0, s>>>(buf); });
  run("empty 1024 x 512", [&] { empty_k<512><<<1024, 512, 0, s>>>(buf); });
  run("empty 2048 x 256", [&] { empty_k<256><<<2048, 256, 0, s>>>(buf); });
  run("touch  256 x 512 (1 MB)", [&] { touch_k<512><<<256, 512, 0, s>>>(buf); });
  run("touch 2048 x 512 (8 MB)", [&] { touch_k<512><<<2048, 512, 0, s>>>(buf); });
  run("memcpy D2D 8 B", [&] { CK(hipMemcpyAsync(buf, buf + 1000, 8, hipMemcpyDeviceToDevice, s)); });
  run("memset 8 KB", [&] { CK(hipMemsetAsync(buf, 0, 8192, s)); });
  return 0;
}
