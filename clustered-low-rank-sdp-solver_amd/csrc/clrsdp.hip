// clrsdp.hip -- device-resident interior-point iteration behind the C ABI of include/clrsdp.h.
//
// One process drives one GPU.  The handle owns every device buffer; constraint data is uploaded
// once and stays resident.  A loop body of solverank1sdp (MPMP.jl:755-887) is a fixed sequence
// of batched launches on one stream (see DESIGN.md for the stage -> kernel table); the only
// host synchronisation is the final read-back of the iteration statistics.  With
// world_size > 1 each rank owns a subset of clusters and the few cross-cluster quantities (Q,
// the n_y-vectors p and sum_j B_j^T S_j^-1 r_j, and ~10 scalars) are all-gathered through the
// registered exchange and reduced in rank order, so every rank computes identical y, dy, alpha.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <string>
#include <array>
#include <vector>

#include "../../include/clrsdp.h"
#include "kernels.h"
#include "kernels_dense.h"

using namespace clrsdp;
using mw::dd;
using mw::qd;
using mw::Num;

namespace {

std::string g_last_error;

struct ClrsdpError {
  int code;
  std::string msg;
};

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess)                                                           \
      throw ClrsdpError{CLRSDP_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

// zero-filled device allocation; the fill is complete on return (null stream, synchronised:
// no caller has to order it against its own non-blocking streams)
template <class X>
X* dmalloc(size_t n) {
  if (n == 0) n = 1;
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, n * sizeof(X)));
  HIPCHK(hipMemsetAsync(p, 0, n * sizeof(X), nullptr));
  HIPCHK(hipStreamSynchronize(nullptr));
  return reinterpret_cast<X*>(p);
}

// the calling thread's current device, set for the scope and restored after (the C ABI's calls
// are made from threads that may drive other devices)
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) HIPCHK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// ---------------- RCCL, loaded at run time (the library itself has no link dependency on it,
// so a single-GPU or CPU-side user never needs librccl).  Only the five entry points the
// exchange uses are resolved.
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
};

const Rccl& rccl() {
  static Rccl api;
  static bool tried = false;
  static std::string why;
  if (!tried) {
    tried = true;
    void* so = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((so = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!so) {
      why = std::string("cannot load librccl: ") + dlerror();
    } else {
      api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(so, "ncclGetUniqueId"));
      api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(so, "ncclCommInitRank"));
      api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(so, "ncclAllGather"));
      api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(so, "ncclCommDestroy"));
      api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(so, "ncclGetErrorString"));
      api.comm_count = reinterpret_cast<decltype(api.comm_count)>(dlsym(so, "ncclCommCount"));
      if (!api.get_unique_id || !api.comm_init_rank || !api.all_gather || !api.comm_destroy ||
          !api.error_string) {
        api = Rccl{};
        why = "librccl lacks an nccl* entry point";
      }
    }
  }
  if (!api.all_gather) throw ClrsdpError{CLRSDP_E_EXCHANGE, why};
  return api;
}

#define RCCLCHK(x)                                                                       \
  do {                                                                                   \
    ncclResult_t r_ = (x);                                                               \
    if (r_ != ncclSuccess)                                                               \
      throw ClrsdpError{CLRSDP_E_EXCHANGE, std::string(#x) + ": " + rccl().error_string(r_)}; \
  } while (0)

template <class X>
X* upload_vec(const std::vector<X>& v) {
  X* p = dmalloc<X>(v.size());
  if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(X), hipMemcpyHostToDevice));
  return p;
}

inline unsigned cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) applies to the current device only: `seen` is
// the caller's per-kernel bitmask of the devices it was already set on
inline void lds_attr_once(std::atomic<unsigned long long>& seen, const void* fn, int bytes) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  const unsigned long long bit = 1ull << (dev & 63);
  if (seen.load(std::memory_order_acquire) & bit) return;
  HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  seen.fetch_or(bit, std::memory_order_acq_rel);
}

// --------------------------------------------------------------------------------------------
// launch plans: descriptor arrays built once at creation, replayed every iteration
// --------------------------------------------------------------------------------------------
// register-tile shapes of chol_inv_reg per word type (NMAX = TR * GR)
template <class T> struct RegCfg { static constexpr int TR = 4, TC = 8, GR = 32, GC = 16; };
template <> struct RegCfg<dd> { static constexpr int TR = 1, TC = 4, GR = 64, GC = 16; };  // 1024 threads
template <> struct RegCfg<qd> { static constexpr int TR = 1, TC = 1, GR = 32, GC = 32; };  // 1024 threads
// chol_lookahead's switches (CLRSDP_LA_OPTS, kernels_dense.h).  Default 2: one Newton step for
// the quad-double pivot reciprocal (~2^-208 relative; the second step was a third of the chain:
// C5 879 -> 930 it/s, round 5 A/B); bit 0 (chain priority) measured nothing
// Only bits 0 and 1 exist; any other value of CLRSDP_LA_OPTS (not a number, other bits) is
// rejected with a message and the default kept.
inline int la_opts() {
  static const int o = [] {
    const char* e = std::getenv("CLRSDP_LA_OPTS");
    if (!e) return 2;
    char* end = nullptr;
    const long v = std::strtol(e, &end, 10);
    if (end == e || *end != '\0' || v < 0 || (v & ~3L)) {
      std::fprintf(stderr, "clrsdp: CLRSDP_LA_OPTS=%s ignored (bits 0 and 1 only); using 2\n", e);
      return 2;
    }
    return (int)v;
  }();
  return o;
}
template <class T> constexpr int reg_nmax() { return std::is_same<T, double>::value ? 128 : RegCfg<T>::TR * RegCfg<T>::GR; }
// multi-word blocks n <= 64 factor with chol_packed (liveness-packed slots, bitwise the same
// factors as chol_inv_reg); CLRSDP_CHOL_PACKED=0 keeps the tile grid (A/B)
inline bool chol_packed_on() {
  static const bool on = [] {
    const char* e = std::getenv("CLRSDP_CHOL_PACKED");
    return !(e && e[0] == '0');
  }();
  return on;
}
// quad-double factors in the square-root-free form (chol_packed LDL); CLRSDP_CHOL_LDL=0: LL^T
inline bool chol_ldl_on() {
  static const bool on = [] {
    const char* e = std::getenv("CLRSDP_CHOL_LDL");
    return !(e && e[0] == '0');
  }();
  return on;
}
template <class T, bool INV, int NMAX = 64>
void launch_chol_packed(unsigned nb, hipStream_t s, const MatDesc<T>* in, const MatDesc<T>* oi,
                        const MatDesc<T>* ol, int* info) {
  constexpr int NT = 1024;
  if constexpr (std::is_same<T, mw::qd>::value) {
    if (chol_ldl_on()) {
      chol_packed<T, NT, INV, true, NMAX><<<nb, NT, 0, s>>>(in, oi, ol, info);
      return;
    }
  }
  chol_packed<T, NT, INV, false, NMAX><<<nb, NT, 0, s>>>(in, oi, ol, info);
}
// eigmin_lds: A (n^2), v, NC = 8 (n <= 64) or 4 partial vectors, dg, e2, w, scalars
template <class T> size_t eig_lds_bytes(int n) {
  return sizeof(T) * ((size_t)n * n + (n <= 64 ? 14 : 10) * (size_t)n + 40);
}
constexpr size_t LDS_MAX = 160 * 1024;

// workgroup order for a batched launch: tile-major, problem fastest (see TileRef)
inline std::vector<TileRef> tile_major(const std::vector<int>& ntiles) {
  std::vector<TileRef> out;
  int mx = 0;
  for (int n : ntiles) mx = std::max(mx, n);
  for (int t = 0; t < mx; ++t)
    for (size_t p = 0; p < ntiles.size(); ++p)
      if (t < ntiles[p]) out.push_back(TileRef{(int)p, t});
  return out;
}

// a development switch is on when set to anything but a value starting with '0' (so that
// NAME=0 switches it off again, for every switch alike)
static inline bool env_on(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] != '0';
}
// a default-on switch is off only when set to a value starting with '0'
static inline bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '0';
}

// work enqueued on another stream for one scope: `stream` is restored when the scope ends,
// also when a launch inside throws (a capture-abort path relies on `stream` being the main one)
struct StreamSwitch {
  hipStream_t& cur;
  hipStream_t saved;
  StreamSwitch(hipStream_t& c, hipStream_t to) : cur(c), saved(c) { cur = to; }
  ~StreamSwitch() { cur = saved; }
  StreamSwitch(const StreamSwitch&) = delete;
  StreamSwitch& operator=(const StreamSwitch&) = delete;
};

// the plans own their device descriptor arrays (freed with the plan; plans are never copied)
struct PlanBase {
  std::vector<void*> owned_dev;
  PlanBase() = default;
  PlanBase(const PlanBase&) = delete;
  PlanBase& operator=(const PlanBase&) = delete;
  ~PlanBase() {
    for (void* p : owned_dev) (void)hipFree(p);
  }
  template <class X>
  X* own(const std::vector<X>& v) {
    X* p = upload_vec(v);
    owned_dev.push_back(p);
    return p;
  }
};

template <class T>
struct GemmPlan : PlanBase {
  bool ta = false, tb = false;
  int tag = 0;  // 1: the Schur-stage V^T X^-1 / V^T Y launch (named separately in profiles)
  unsigned long long* stamp = nullptr;  // tag 1: earliest workgroup start (SCHUR timing)
  std::vector<GemmDesc<T>> h;
  std::vector<int> ntiles;  // per problem
  std::vector<TileRef> t2d;
  GemmDesc<T>* d = nullptr;
  TileRef* dt = nullptr;
  // gemm_f64_lds (fp64) and gemm_valu_ks (multi-word; CLRSDP_GEMM_VALU16=1: gemm_valu) output
  // tiles, fixed when the plan is created
  const int TILE = std::is_same<T, double>::value ? 64 : env_on("CLRSDP_GEMM_VALU16") ? 16 : 8;

  void clear() {  // back to an empty plan (a failed build_lu_plans)
    h.clear();
    ntiles.clear();
    t2d.clear();
    d = nullptr;
    dt = nullptr;
  }
  void add(const T* A, int lda, const T* B, int ldb, const T* Cin, int ldcin, T* C, int ldc, int M,
           int N, int K) {
    if (M <= 0 || N <= 0) return;
    GemmDesc<T> g;
    g.A = A; g.B = B; g.Cin = Cin; g.C = C;
    g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldcin = ldcin; g.ldc = ldc;
    g.tn = cdiv(N, TILE);
    g.tile0 = 0;
    g.flags = 0;
    g.alpha = g.beta = 0.0;
    g.sa = g.sl = nullptr;
    ntiles.push_back((int)(cdiv(M, TILE) * g.tn));
    h.push_back(g);
  }
  // sca: op(A) = A with column k scaled by sa[k] * sl[k] (fp64, NT: the weighted-A products)
  bool sca = false;
  void add_scaled(const T* A, int lda, const T* B, int ldb, const T* Cin, int ldcin, T* C, int ldc,
                  int M, int N, int K, const T* sa, const T* sl) {
    if (M <= 0 || N <= 0) return;
    sca = true;
    add(A, lda, B, ldb, Cin, ldcin, C, ldc, M, N, K);
    h.back().sa = sa;
    h.back().sl = sl;
  }
  // dyn: a mixed batch (fp64): op(A), op(B), alpha and beta per problem (gemm_f64_dyn)
  bool dyn = false;
  void add_op(bool opa, bool opb, double al, double be, const T* A, int lda, const T* B, int ldb,
              const T* Cin, int ldcin, T* C, int ldc, int M, int N, int K) {
    if (M <= 0 || N <= 0) return;
    dyn = true;
    add(A, lda, B, ldb, Cin, ldcin, C, ldc, M, N, K);
    h.back().flags = (opa ? 1 : 0) | (opb ? 2 : 0) | 4;
    h.back().alpha = al;
    h.back().beta = be;
  }
  bool gemv = false;
  // sym: every problem square with an exactly symmetric result wanted (gemm_f64_lds SYM: the
  // lower tiles only, each written with its mirror image); fp64, beta = 0
  bool sym = false;
  // prio: raised wave priority for a critical-path batch that runs beside side-stream work
  // (gemm_f64_uni / gemm_f64_dyn; set before finalize)
  bool prio = false;
  // upper (multi-word, round 6): every problem square with a symmetric product of which only the
  // tiles on and above the diagonal are wanted (the Schur pairings V^T X^-1 V, V^T Y V of m = 1
  // blocks: schur_assemble reads (min, max)); the launch lists those tiles only -- half the
  // VALU-bound multi-word work
  bool upper = false;
  void finalize() {
    if (h.empty()) return;
    if (sca && (ta || !tb || !std::is_same<T, double>::value))
      throw ClrsdpError{CLRSDP_E_ARG, "scaled-A GEMM: fp64 A B^T only"};
    gemv = !dyn && !sca;  // (a mixed or scaled batch always takes the tiled kernel)
    for (const auto& g : h) gemv = gemv && g.N == 1;
    // op(B) = B^T of a 1 x K row is the gemv vector only for K = 1 (e.g. all blocks 1 x 1)
    if (gemv && tb)
      for (const auto& g : h) gemv = gemv && g.K == 1;
    if (gemv) sym = false;  // a product with one column is 1 x 1 when square: trivially symmetric
    if (gemv)  // one workgroup per 64 outputs
      for (size_t q = 0; q < h.size(); ++q) ntiles[q] = (int)cdiv(h[q].M, 64);
    if (dyn && (gemv || sym || !std::is_same<T, double>::value))
      throw ClrsdpError{CLRSDP_E_ARG, "mixed GEMM batch: fp64 matrices only"};
    if (sym) {
      if (gemv || !std::is_same<T, double>::value)
        throw ClrsdpError{CLRSDP_E_ARG, "symmetric GEMM epilogue: fp64 matrices only"};
      for (const auto& g : h)
        if (g.M != g.N) throw ClrsdpError{CLRSDP_E_ARG, "symmetric GEMM epilogue: square problems only"};
      // tile-major over the lower tiles (tm >= tn) of each problem, problem fastest
      int mx = 0;
      for (int n : ntiles) mx = std::max(mx, n);
      for (int t = 0; t < mx; ++t)
        for (size_t p = 0; p < h.size(); ++p)
          if (t < ntiles[p] && t / h[p].tn >= t % h[p].tn) t2d.push_back(TileRef{(int)p, t});
    } else if (upper && !gemv && !std::is_same<T, double>::value) {
      int mx = 0;
      for (int n : ntiles) mx = std::max(mx, n);
      for (int t = 0; t < mx; ++t)
        for (size_t p = 0; p < h.size(); ++p)
          if (t < ntiles[p] && t / h[p].tn <= t % h[p].tn) t2d.push_back(TileRef{(int)p, t});
    } else {
      t2d = tile_major(ntiles);
    }
    if (prio && dyn)
      for (auto& g : h) g.flags |= 8;
    d = own(h);
    dt = own(t2d);
    detect_uniform();
    ug.prio = prio ? 1 : 0;
  }
  // fp64 batches of one shape at constant operand strides take gemm_f64_uni (no descriptor
  // chain before the first operand load); CLRSDP_NO_UNI_GEMM keeps the descriptor kernels
  bool uni = false;
  int uts = 64;  // gemm_f64_uni output tile (64 or 32)
  UniGemm ug{};
  void detect_uniform() {
    if constexpr (std::is_same<T, double>::value) {
      static const bool off = env_on("CLRSDP_NO_UNI_GEMM");
      if (off || gemv || dyn || h.empty()) return;
      const GemmDesc<T>& g0 = h[0];
      auto stride = [&](auto get, long long& st) {
        st = h.size() > 1 ? (long long)(get(h[1]) - get(h[0])) : 0;
        for (size_t p = 1; p < h.size(); ++p)
          if ((long long)(get(h[p]) - get(h[p - 1])) != st) return false;
        return true;
      };
      for (const auto& g : h)
        if (g.M != g0.M || g.N != g0.N || g.K != g0.K || g.lda != g0.lda || g.ldb != g0.ldb ||
            g.ldc != g0.ldc || g.ldcin != g0.ldcin || (g.Cin == nullptr) != (g0.Cin == nullptr) ||
            (g.sa == nullptr) != (g0.sa == nullptr))
          return;
      UniGemm u{};
      bool ok = stride([](const GemmDesc<T>& g) { return g.A; }, u.sA) &&
                stride([](const GemmDesc<T>& g) { return g.B; }, u.sB) &&
                stride([](const GemmDesc<T>& g) { return (const T*)g.C; }, u.sC);
      if (g0.Cin) ok = ok && stride([](const GemmDesc<T>& g) { return g.Cin; }, u.sCin);
      if (g0.sa) ok = ok && stride([](const GemmDesc<T>& g) { return g.sa; }, u.sSa) &&
                      stride([](const GemmDesc<T>& g) { return g.sl; }, u.sSl);
      if (!ok) return;
      u.A = g0.A; u.B = g0.B; u.Cin = g0.Cin; u.C = g0.C; u.sa = g0.sa; u.sl = g0.sl;
      u.M = g0.M; u.N = g0.N; u.K = g0.K; u.lda = g0.lda; u.ldb = g0.ldb; u.ldcin = g0.ldcin;
      u.P = (int)h.size();
      u.ldc = g0.ldc;
      // 32x32 tiles when the 64x64 tiles would leave most CUs idle (a small batch: one CU's
      // tile is then latency-bound, ~9.4 us for a 128^3 product against 6.5 us split over four
      // CUs, tools/micro/gemm_tiles.hip); CLRSDP_GEMM_TS32_BELOW sets the threshold (tiles)
      // (read at every plan build, so a test can force either tile in one process)
      const char* e32 = std::getenv("CLRSDP_GEMM_TS32_BELOW");
      const long ts32_below = e32 ? std::atol(e32) : 192L;
      const long t64m = (long)cdiv(g0.M, 64), t64n = (long)cdiv(g0.N, 64);
      const long tiles64 = u.P * (sym ? t64m * (t64m + 1) / 2 : t64m * t64n);
      uts = tiles64 < ts32_below ? 32 : 64;
      u.tn = (int)cdiv(g0.N, uts);
      const int tm = (int)cdiv(g0.M, uts);
      u.tsym = tm * (tm + 1) / 2;
      ug = u;
      uni = true;
    }
  }
  template <class U = T>
  void launch_uni_impl(hipStream_t s, double alpha, double beta, const double* ds, double dmult) const;
  void launch_uni(hipStream_t s, double alpha, double beta, const double* ds, double dmult) const {
    launch_uni_impl<T>(s, alpha, beta, ds, dmult);
  }
  // C = alpha op(A) op(B) + beta Cin (+ dmult * *dscal on the diagonal of square problems)
  void launch(hipStream_t s, double alpha, double beta, const T* dscal = nullptr,
              double dmult = 0.0) const {
    if (h.empty()) return;
    if (dscal && !std::is_same<T, double>::value)
      throw ClrsdpError{CLRSDP_E_ARG, "fused diagonal epilogue is fp64 only"};
    const unsigned grid = (unsigned)t2d.size();
    if (gemv) {  // (tb only with K = 1: B[0] is the vector either way)
      // fp64: deep load pipelines (CLRSDP_GEMV_DEEP=0: the 8-deep round-4 loops)
      // (multi-word, transposed: DEEP selects the thread-per-column form, the quad-double default
      // -- C5 936 -> 977 it/s; double-double keeps the 16-lane reduction form, 834 against 820
      // with the column form -- CLRSDP_GEMV_MW_T16=1 / CLRSDP_GEMV_MW_COL=1 swap them; round 5)
      static const bool deep = !env_off("CLRSDP_GEMV_DEEP");
      static const bool mw_t16 = env_on("CLRSDP_GEMV_MW_T16"), mw_col = env_on("CLRSDP_GEMV_MW_COL");
      const bool deep_t = std::is_same<T, double>::value ? deep
                          : std::is_same<T, mw::qd>::value ? !mw_t16
                                                           : mw_col;
      if (ta && deep_t) gemv_batched<T, true><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else if (ta) gemv_batched<T, true, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else if (deep) gemv_batched<T, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else gemv_batched<T, false, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      HIPCHK(hipGetLastError());
      return;
    }
    if constexpr (std::is_same<T, double>::value) {
      const double* ds = reinterpret_cast<const double*>(dscal);
      if (uni) {
        launch_uni(s, alpha, beta, ds, dmult);
        return;
      }
      if (sca) {
        gemm_f64_lds<false, true, 0, 32, 8, false, true><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult);
        HIPCHK(hipGetLastError());
        return;
      }
      if (dyn) {  // alpha/beta come from the descriptors
        gemm_f64_dyn<><<<grid, 512, 0, s>>>(d, dt, alpha, beta);
        HIPCHK(hipGetLastError());
        return;
      }
      if (sym) {
        if (beta != 0.0 || ds) throw ClrsdpError{CLRSDP_E_ARG, "symmetric GEMM epilogue: beta = 0 only"};
        if (!ta && tb) gemm_f64_lds<false, true, 0, 32, 8, true><<<grid, 512, 0, s>>>(d, dt, alpha, 0.0);
        else if (!ta && !tb) gemm_f64_lds<false, false, 0, 32, 8, true><<<grid, 512, 0, s>>>(d, dt, alpha, 0.0);
        else throw ClrsdpError{CLRSDP_E_ARG, "symmetric GEMM epilogue: op(A) = A only"};
        HIPCHK(hipGetLastError());
        return;
      }
      if (tag == 1 && !ta && tb) gemm_f64_lds<false, true, 1><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult, stamp);
      else if (tag == 3 && !ta && tb) gemm_f64_lds<false, true, 3><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult, stamp);
      else if (!ta && !tb) gemm_f64_lds<false, false><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult);
      else if (ta && !tb) gemm_f64_lds<true, false><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult);
      else if (!ta && tb) gemm_f64_lds<false, true><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult);
      else gemm_f64_lds<true, true><<<grid, 512, 0, s>>>(d, dt, alpha, beta, ds, dmult);
    } else if (TILE == 8) {
      if (!ta && !tb) gemm_valu_ks<T, false, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else if (ta && !tb) gemm_valu_ks<T, true, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else if (!ta && tb) gemm_valu_ks<T, false, true><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else gemm_valu_ks<T, true, true><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
    } else {
      if (!ta && !tb) gemm_valu<T, false, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else if (ta && !tb) gemm_valu<T, true, false><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else if (!ta && tb) gemm_valu<T, false, true><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
      else gemm_valu<T, true, true><<<grid, 256, 0, s>>>(d, dt, alpha, beta);
    }
    HIPCHK(hipGetLastError());
  }
};

// Two dependent products of every block as one launch by column strips (chain_f64, fp64,
// uniform n x n blocks with n <= 128): T = a1 A1 op(B1)[:, S] + b1 C1[:, S], O[:, S] = A2 T
struct ChainPlan {
  bool on = false, tb1 = false, sym = false, trace = false;
  ChainGemm u{};
  // one pointer set per arena; the blocks sit at stride n^2 (checked by the caller)
  void set(int half, const double* A1, const double* B1, const double* C1, const double* A2,
           double* O) {
    u.A1[half] = A1; u.B1[half] = B1; u.C1[half] = C1; u.A2[half] = A2; u.O[half] = O;
  }
  void init(int n, int nb, int halves, bool tb, bool sy) {
    on = true;
    tb1 = tb;
    sym = sy;
    u.n = n;
    u.lda1 = u.ldb1 = u.ldc1 = u.lda2 = u.ldo = n;
    u.sA1 = u.sB1 = u.sC1 = u.sA2 = u.sO = (long long)n * n;
    u.P1 = nb;
    u.P = nb * halves;
    if (halves == 1) set(1, nullptr, nullptr, nullptr, nullptr, nullptr);
    for (const void* k : {(const void*)chain_f64<false, false>, (const void*)chain_f64<true, true>,
                          (const void*)chain_f64<false, false, true>})
      HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chain::LDS));
  }
  void launch(hipStream_t s, double a1, double b1) const {
    const unsigned grid = (unsigned)(u.P * (int)cdiv(trace ? u.NC : u.n, chain::NS));
    if (trace) chain_f64<false, false, true><<<grid, 512, chain::LDS_TRACE, s>>>(u, a1, b1);
    else if (tb1 && sym) chain_f64<true, true><<<grid, 512, chain::LDS, s>>>(u, a1, b1);
    else if (!tb1 && !sym) chain_f64<false, false><<<grid, 512, chain::LDS, s>>>(u, a1, b1);
    else throw ClrsdpError{CLRSDP_E_ARG, "chain_f64: unsupported variant"};
    HIPCHK(hipGetLastError());
  }
};

template <bool DB, int TS>
void launch_uni_db(const UniGemm& u, hipStream_t s, bool ta, bool tb, bool sca, bool sym, int tag,
                   unsigned long long* stamp, double alpha, double beta, const double* ds, double dmult) {
  constexpr int NW = TS == 64 ? 8 : 2, NT = 64 * NW;
  const unsigned tiles = (unsigned)(u.P * (int)cdiv(u.M, TS) * u.tn);
  if (sca) {
    gemm_f64_uni<false, true, 0, 32, NW, false, true, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult);
  } else if (sym) {
    if (beta != 0.0 || ds) throw ClrsdpError{CLRSDP_E_ARG, "symmetric GEMM epilogue: beta = 0 only"};
    const unsigned grid = (unsigned)(u.P * u.tsym);
    if (!ta && tb) gemm_f64_uni<false, true, 0, 32, NW, true, false, DB, TS><<<grid, NT, 0, s>>>(u, alpha, 0.0);
    else if (!ta && !tb) gemm_f64_uni<false, false, 0, 32, NW, true, false, DB, TS><<<grid, NT, 0, s>>>(u, alpha, 0.0);
    else throw ClrsdpError{CLRSDP_E_ARG, "symmetric GEMM epilogue: op(A) = A only"};
  } else {
    if (tag == 1 && !ta && tb) gemm_f64_uni<false, true, 1, 32, NW, false, false, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult, stamp);
    else if (tag == 3 && !ta && tb) gemm_f64_uni<false, true, 3, 32, NW, false, false, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult, stamp);
    else if (!ta && !tb) gemm_f64_uni<false, false, 0, 32, NW, false, false, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult);
    else if (ta && !tb) gemm_f64_uni<true, false, 0, 32, NW, false, false, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult);
    else if (!ta && tb) gemm_f64_uni<false, true, 0, 32, NW, false, false, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult);
    else gemm_f64_uni<true, true, 0, 32, NW, false, false, DB, TS><<<tiles, NT, 0, s>>>(u, alpha, beta, ds, dmult);
  }
  HIPCHK(hipGetLastError());
}

template <class T>
template <class U>
void GemmPlan<T>::launch_uni_impl(hipStream_t s, double alpha, double beta, const double* ds, double dmult) const {
  if constexpr (std::is_same<T, double>::value) {
    // CLRSDP_UNI_DB=0: single-buffered slabs (two barriers per k-step), for A/B timing
    static const bool db = [] {
      const char* e = std::getenv("CLRSDP_UNI_DB");
      return !(e && e[0] == '0');
    }();
    if (uts == 32) launch_uni_db<true, 32>(ug, s, ta, tb, sca, sym, tag, stamp, alpha, beta, ds, dmult);
    else if (db) launch_uni_db<true, 64>(ug, s, ta, tb, sca, sym, tag, stamp, alpha, beta, ds, dmult);
    else launch_uni_db<false, 64>(ug, s, ta, tb, sca, sym, tag, stamp, alpha, beta, ds, dmult);
  }
}

template <class T>
struct TrsmPlan : PlanBase {
  // NC: right-hand sides per workgroup.  Multi-word solves with many right-hand sides
  // (W = L^-1 B) take 16 (one diagonal pass of 256 threads, and four times the workgroups of 64:
  // the panel update's multi-word products spread over more CUs); CLRSDP_TRSM_NC64=1 keeps 64.
  static constexpr int NB = 16, NCW = 64, NCN = 16;
  std::vector<TrsmDesc<T>> h;
  std::vector<int> t2d;
  TrsmDesc<T>* d = nullptr;
  int* dt = nullptr;
  int nmax = 0, rmax = 0;
  bool narrow = false;
  // multi-word solves with n <= 64: trsv_wave, one wave per right-hand side, 4 waves per
  // workgroup for vector solves and 16 (four per SIMD, their chains interleaved; one LDS copy of
  // L per 16 right-hand sides) for W_j = L_j^-1 B_j (CLRSDP_TRSV_BLOCKED=1 keeps trsm_batched)
  static constexpr int NCV = 4, NCV16 = 16;
  bool vec = false;
  int ncv = NCV;
  bool four = false;  // four right-hand sides per workgroup whatever their number (latency first)
  // ident: the right-hand sides are the columns of the identity (L^-1 = L \ I); src: read them
  // from src (ld ldb) and write the solution to B.  Both only in the vector-solve kernels
  // (vec_rhs() after finalize); otherwise the caller fills B first.
  void add(const T* L, int ldl, T* B, int ldb, int n, int nrhs, bool ident = false,
           const T* src = nullptr) {
    if (n <= 0 || nrhs <= 0) return;
    rmax = std::max(rmax, nrhs);
    TrsmDesc<T> t;
    t.L = L; t.B = B; t.n = n; t.nrhs = nrhs; t.ldl = ldl; t.ldb = ldb;
    t.tile0 = 0;
    t.pad = ident ? 1 : 0;
    t.src = src;
    h.push_back(t);
    nmax = std::max(nmax, n);
  }
  void finalize() {
    if (h.empty()) return;
    narrow = mode == 0 && !std::is_same<T, double>::value && rmax >= 32 && !env_on("CLRSDP_TRSM_NC64");
    // (64 < n <= 128: trsv_wave128, L through LDS in 32-step chunks; CLRSDP_TRSV128=0 keeps
    // trsm_batched there)
    const char* e128 = std::getenv("CLRSDP_TRSV128");
    vec = mode == 0 && !std::is_same<T, double>::value && !env_on("CLRSDP_TRSV_BLOCKED") &&
          (nmax <= 64 || (nmax <= 128 && !(e128 && e128[0] == '0')));
    // (CLRSDP_TRSV_NW4=1: four right-hand sides per workgroup whatever their number: one chain
    // per SIMD, more workgroups)
    static const bool nw4 = env_on("CLRSDP_TRSV_NW4");
    ncv = (rmax <= NCV || nw4 || four) ? NCV : NCV16;
    const int nc = vec ? ncv : narrow ? NCN : NCW;
    if constexpr (!std::is_same<T, double>::value) {
      if (vec) {  // (outside any graph capture)
        static std::atomic<unsigned long long> a128[8], a64[8];
        lds_attr_once(a128[0], (const void*)trsv_wave128<T, true, NCV>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[1], (const void*)trsv_wave128<T, false, NCV>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[2], (const void*)trsv_wave128<T, true, NCV16>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[3], (const void*)trsv_wave128<T, false, NCV16>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[4], (const void*)trsv_wave128<T, true, NCV, false>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[5], (const void*)trsv_wave128<T, false, NCV, false>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[6], (const void*)trsv_wave128<T, true, NCV16, false>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a128[7], (const void*)trsv_wave128<T, false, NCV16, false>, (int)trsv_wave128_lds<T>());
        lds_attr_once(a64[0], (const void*)trsv_wave<T, true, NCV>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[1], (const void*)trsv_wave<T, false, NCV>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[2], (const void*)trsv_wave<T, true, NCV16>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[3], (const void*)trsv_wave<T, false, NCV16>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[4], (const void*)trsv_wave<T, true, NCV, false>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[5], (const void*)trsv_wave<T, false, NCV, false>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[6], (const void*)trsv_wave<T, true, NCV16, false>, (int)trsv_wave_lds<T>());
        lds_attr_once(a64[7], (const void*)trsv_wave<T, false, NCV16, false>, (int)trsv_wave_lds<T>());
      }
    }
    if (!vec_rhs())
      for (TrsmDesc<T>& t : h) { t.pad = 0; t.src = nullptr; }  // (the caller fills B)
    t2d.clear();
    for (size_t q = 0; q < h.size(); ++q) {
      h[q].tile0 = (int)t2d.size();
      for (int i = 0; i < (int)cdiv(h[q].nrhs, nc); ++i) t2d.push_back((int)q);
    }
    d = own(h);
    dt = own(t2d);
  }
  template <bool PF>
  void launch_vec(hipStream_t s, bool trans, unsigned grid) const {
    if constexpr (!std::is_same<T, double>::value) {
      if (nmax > 64) {
        const size_t l = trsv_wave128_lds<T>();
        if (ncv == NCV16) {
          if (trans) trsv_wave128<T, true, NCV16, PF><<<grid, 64 * NCV16, l, s>>>(d, dt);
          else trsv_wave128<T, false, NCV16, PF><<<grid, 64 * NCV16, l, s>>>(d, dt);
        } else {
          if (trans) trsv_wave128<T, true, NCV, PF><<<grid, 64 * NCV, l, s>>>(d, dt);
          else trsv_wave128<T, false, NCV, PF><<<grid, 64 * NCV, l, s>>>(d, dt);
        }
      } else if (ncv == NCV16) {
        if (trans) trsv_wave<T, true, NCV16, PF><<<grid, 64 * NCV16, trsv_wave_lds<T>(), s>>>(d, dt);
        else trsv_wave<T, false, NCV16, PF><<<grid, 64 * NCV16, trsv_wave_lds<T>(), s>>>(d, dt);
      } else {
        if (trans) trsv_wave<T, true, NCV, PF><<<grid, 64 * NCV, trsv_wave_lds<T>(), s>>>(d, dt);
        else trsv_wave<T, false, NCV, PF><<<grid, 64 * NCV, trsv_wave_lds<T>(), s>>>(d, dt);
      }
    }
  }
  // the vector-solve kernels take the identity / a separate source as right-hand sides
  // (CLRSDP_TRSV_RHS=0: the caller copies them into B, as before round 6)
  bool vec_rhs() const {
    static const bool on = !env_off("CLRSDP_TRSV_RHS");
    return on && vec && mode == 0 && !std::is_same<T, double>::value;
  }
  // mode (the LU fallback's factors): 0 = potrf's L; 1 = unit lower L of getrf; 2 = getrf's U,
  // read transposed (forward: U^T x = b; trans: U x = b)
  int mode = 0;
  void launch(hipStream_t s, bool trans) const {
    if (h.empty()) return;
    constexpr int NC = NCW;
    const size_t lds = sizeof(T) * ((size_t)NB * NB + (size_t)NB * NC + (size_t)NB * nmax);
    const unsigned grid = (unsigned)t2d.size();
    if constexpr (!std::is_same<T, double>::value) {
      if (vec && mode == 0) {
        // (CLRSDP_TRSV_PF=0: the staging loops that wait on each load of L in turn)
        static const bool pf = !env_off("CLRSDP_TRSV_PF");
        if (pf) launch_vec<true>(s, trans, grid);
        else launch_vec<false>(s, trans, grid);
        HIPCHK(hipGetLastError());
        return;
      }
    }
    if (narrow && mode == 0) {
      const size_t ldsn = sizeof(T) * ((size_t)NB * NB + (size_t)NB * NCN + (size_t)NB * nmax);
      if (trans) trsm_batched<T, true, NB, NCN, 256><<<grid, 256, ldsn, s>>>(d, dt);
      else trsm_batched<T, false, NB, NCN, 256><<<grid, 256, ldsn, s>>>(d, dt);
      HIPCHK(hipGetLastError());
      return;
    }
    if (mode == 1 && !trans) {
      trsm_batched<T, false, NB, NC, 256, true, false><<<grid, 256, lds, s>>>(d, dt);
      HIPCHK(hipGetLastError());
      return;
    }
    if (mode == 2) {
      if (trans) trsm_batched<T, true, NB, NC, 256, false, true><<<grid, 256, lds, s>>>(d, dt);
      else trsm_batched<T, false, NB, NC, 256, false, true><<<grid, 256, lds, s>>>(d, dt);
      HIPCHK(hipGetLastError());
      return;
    }
    if (mode != 0) throw ClrsdpError{CLRSDP_E_ARG, "unsupported triangular solve mode"};
    // multi-word solves with many right-hand sides (W = L^-1 B): 1024 threads, four waves per
    // SIMD for the VALU-bound panel update; vector solves keep 256
    if (!std::is_same<T, double>::value && rmax >= 32) {
      if (trans) trsm_batched<T, true, NB, NC, 1024><<<grid, 1024, lds, s>>>(d, dt);
      else trsm_batched<T, false, NB, NC, 1024><<<grid, 1024, lds, s>>>(d, dt);
    } else {
      if (trans) trsm_batched<T, true, NB, NC><<<grid, 256, lds, s>>>(d, dt);
      else trsm_batched<T, false, NB, NC><<<grid, 256, lds, s>>>(d, dt);
    }
    HIPCHK(hipGetLastError());
  }
};

template <class T>
struct MatPlan : PlanBase {  // potrf / eigmin
  static constexpr int NB = 16;
  std::vector<MatDesc<T>> h;
  MatDesc<T>* d = nullptr;
  int nmax = 0;
  void add(T* A, int n, int lda) {
    MatDesc<T> m;
    m.A = A; m.n = n; m.lda = lda;
    h.push_back(m);
    nmax = std::max(nmax, n);
  }
  // multi-word Cholesky factors of blocks with n <= 128: the register-resident chol_packed
  // without the inverse (1024 threads, the whole block on chip, two barriers per column) writes
  // L in place -- against potrf_batched's 16-column panels with a serial pivot chain (n <= 64
  // falls back to chol_inv_reg with CLRSDP_CHOL_PACKED=0).  Set before finalize();
  // CLRSDP_REG_POTRF=0 keeps potrf_batched.
  bool reg_potrf = false;
  int* redo = nullptr;  // eigmin_mx's per-block fallback flags
  // blocked multi-word potrf across workgroups (potrf_blk_*, kernels_dense.h; round 6): taken
  // for the double-double blocks above 64 (CLRSDP_POTRF_BLK=0 keeps chol_lookahead there).
  // 16-column panels: n = 127 x 16 blocks 230 -> 155 us (32-column panels: 201 us), while at
  // n <= 64 the one-CU chol_lookahead stays ahead (52 against 73 us; tools/micro/potrf_blk_bench)
  static constexpr int BLK_NB = 16;
  BlkPotrfDesc<T>* bd = nullptr;
  bool blk = false;
  void finalize() {
    if (h.empty()) return;
    d = own(h);
    if constexpr (std::is_same<T, mw::dd>::value) {
      blk = nmax > 64 && !env_off("CLRSDP_POTRF_BLK");
      if (blk) {
        T* li = own(std::vector<T>(h.size() * BLK_NB * BLK_NB, T(0.0)));
        std::vector<BlkPotrfDesc<T>> b(h.size());
        for (size_t q = 0; q < h.size(); ++q)
          b[q] = BlkPotrfDesc<T>{h[q].A, li + q * BLK_NB * BLK_NB, h[q].n, h[q].lda};
        bd = own(b);
      }
    }
    if (!std::is_same<T, double>::value) redo = own(std::vector<int>(h.size(), 1));
    const char* e = std::getenv("CLRSDP_REG_POTRF");
    // (double-double blocks 65..128: chol_packed only, CLRSDP_CHOL_PACKED128=0 keeps
    // potrf_batched there; quad-double would spill at nine slots per thread)
    const char* e2 = std::getenv("CLRSDP_CHOL_PACKED128");
    const int lim = std::is_same<T, mw::dd>::value && chol_packed_on() && !(e2 && e2[0] == '0') ? 128 : 64;
    reg_potrf = reg_potrf && !std::is_same<T, double>::value && nmax <= lim && !(e && e[0] == '0');
  }
  void potrf(hipStream_t s, int* info) const {
    if (h.empty()) return;
    if constexpr (std::is_same<T, mw::dd>::value) {
      if (blk) {
        constexpr int NB = BLK_NB, DT = NB / 16;
        const unsigned nm = (unsigned)h.size();
        potrf_blk_first<T, false, NB><<<nm, 256, 0, s>>>(bd, info, la_opts());
        for (int k0 = 0; k0 + NB < nmax; k0 += NB) {
          const int rows = nmax - k0 - NB, ntr = cdiv(rows, 16);
          int tiles = 0;  // lower 16-tiles of the trailing matrix outside the next diagonal block
          for (int I = DT; I < ntr; ++I) tiles += I + 1;
          potrf_blk_trsm<T, NB><<<dim3((unsigned)ntr, nm), 256, 0, s>>>(bd, k0);
          potrf_blk_update<T, false, NB><<<dim3(1u + tiles, nm), 256, 0, s>>>(bd, k0, info, la_opts());
        }
        HIPCHK(hipGetLastError());
        return;
      }
    }
    if constexpr (!std::is_same<T, double>::value) {
      // the look-ahead potrf (chol_lookahead: the pivot chain beside the trailing update);
      // CLRSDP_CHOL_LA=0 keeps chol_packed.  At n <= 64 the bulk waves on the chain's SIMD stay
      // idle (SKIP0, round 6: qd n = 51 138 -> 126 us, dd n = 64 63 -> 61 us)
      static const bool la = !env_off("CLRSDP_CHOL_LA");
      if (reg_potrf && la && nmax <= (std::is_same<T, mw::dd>::value ? 128 : 64)) {
        bool done = false;
        if constexpr (std::is_same<T, mw::dd>::value) {  // (no quad-double instance: it would spill)
          if (nmax > 64) {
            chol_lookahead<T, false, false, 128><<<(unsigned)h.size(), 1024, 0, s>>>(d, nullptr, d, info, la_opts());
            done = true;
          }
        }
        if (done) {
        } else if (std::is_same<T, mw::qd>::value && chol_ldl_on())
          chol_lookahead<T, false, true, 64, 15, true><<<(unsigned)h.size(), 1024, 0, s>>>(d, nullptr, d, info, la_opts());
        else
          chol_lookahead<T, false, false, 64, 15, true><<<(unsigned)h.size(), 1024, 0, s>>>(d, nullptr, d, info, la_opts());
        HIPCHK(hipGetLastError());
        return;
      }
      if (reg_potrf) {
        if constexpr (std::is_same<T, mw::dd>::value) {
          if (nmax > 64) {
            chol_packed<T, 1024, false, false, 128><<<(unsigned)h.size(), 1024, 0, s>>>(d, d, d, info);
            HIPCHK(hipGetLastError());
            return;
          }
        }
        if (chol_packed_on())
          launch_chol_packed<T, false>((unsigned)h.size(), s, d, d, d, info);
        else
          chol_inv_reg<T, 1, 4, 64, 16, false><<<(unsigned)h.size(), 1024, 0, s>>>(d, d, d, info);
        HIPCHK(hipGetLastError());
        return;
      }
    }
    const size_t lds = sizeof(T) * ((size_t)NB * NB + (size_t)NB * nmax);
    // double-double: 1024 threads, so the trailing update (VALU bound) has four waves per SIMD
    // (C4 factor stage 806 -> 724 us); quad-double keeps 256 (its registers, 3 % slower at 1024)
    constexpr int NT = std::is_same<T, mw::dd>::value ? 1024 : 256;
    potrf_batched<T, NB, NT><<<(unsigned)h.size(), NT, lds, s>>>(d, info);
    HIPCHK(hipGetLastError());
  }
  void eigmin(hipStream_t s, T* out) const {
    if (h.empty()) return;
    if constexpr (std::is_same<T, double>::value) {
      if (nmax <= 128) {  // matrix in registers
        // eigmin_split (round 4: one reflector chain wave + 8 bulk waves) unless
        // CLRSDP_EIG_REG=1 (eigmin_reg: every live wave builds the reflector)
        static const bool reg = env_on("CLRSDP_EIG_REG");
        // the last 24 columns on the chain wave alone (no barriers): 144.0 against 147.4 us per
        // batch of 128 blocks of 128, bitwise the same lambda_min on 1048 of 1056 test blocks
        // (tools/micro/eig_split_bench.hip); CLRSDP_EIG_TAIL=0 keeps the two-barrier loop
        static const bool etail = !env_off("CLRSDP_EIG_TAIL");
        // (round 6: eigmin_onebar, one barrier per column with the next reflector's
        // matrix-vector product under the chain's reflector, measured 203 against 143 us per
        // batch of 128 blocks of 128 -- the bulk waves are VALU-issue bound -- and stays a
        // microbenchmark, tools/micro/eig_onebar_bench.hip)
        if (reg) eigmin_reg<<<(unsigned)h.size(), 512, 0, s>>>(d, out);
        else if (etail) eigmin_split<0, 24><<<(unsigned)h.size(), 576, 0, s>>>(d, out);
        else eigmin_split<0><<<(unsigned)h.size(), 576, 0, s>>>(d, out);
        HIPCHK(hipGetLastError());
        return;
      }
    }
    // CLRSDP_EIG_NEWTON=0 keeps the multi-word multisection from the fp64 bracket (A/B)
    static const bool newton = [] {
      const char* e = std::getenv("CLRSDP_EIG_NEWTON");
      return !(e && e[0] == '0');
    }();
    // multi-word, n <= 64: an fp64 eigenpair refined at the word's width (eigmin_mx; the blocks
    // it cannot certify go to eigmin_lds2 in a second, flagged launch) unless CLRSDP_EIG_MX=0
    static const bool mx = [] {
      const char* e = std::getenv("CLRSDP_EIG_MX");
      return !(e && e[0] == '0');
    }();
    if constexpr (!std::is_same<T, double>::value) {
      if (mx && newton && redo && nmax <= 64 && eigmx_lds_bytes<T>(nmax) + EIGMX_STATIC_LDS <= LDS_MAX &&
          eig2_lds_bytes<T>(nmax) <= LDS_MAX && (sizeof(T) <= 16 || nmax <= 64)) {
        static std::atomic<unsigned long long> attrm{0}, attr2r{0};
        static const bool dbg = env_on("CLRSDP_EIGMX_STATS");
        if (dbg) {  // (the diagnostics instance: per-block eta / lambda / Temple width)
          static std::atomic<unsigned long long> attrd{0};
          lds_attr_once(attrd, (const void*)eigmin_mx<T, 1>, (int)(LDS_MAX - EIGMX_STATIC_LDS));
          eigmin_mx<T, 1><<<(unsigned)h.size(), 576, eigmx_lds_bytes<T>(nmax), s>>>(d, out, redo);
        } else {
          lds_attr_once(attrm, (const void*)eigmin_mx<T>, (int)(LDS_MAX - EIGMX_STATIC_LDS));
          eigmin_mx<T><<<(unsigned)h.size(), 576, eigmx_lds_bytes<T>(nmax), s>>>(d, out, redo);
        }
        HIPCHK(hipGetLastError());
        // the flagged blocks (clustered lambda_min) at the full width; the others exit at once
        lds_attr_once(attr2r, (const void*)eigmin_lds2<T, true>, (int)LDS_MAX);
        eigmin_lds2<T, true><<<(unsigned)h.size(), 512, eig2_lds_bytes<T>(nmax), s>>>(d, out, redo);
        HIPCHK(hipGetLastError());
        return;
      }
    }
    // multi-word: eigmin_lds2 (two barriers per column) unless CLRSDP_EIG_LDS1=1
    static const bool lds1 = env_on("CLRSDP_EIG_LDS1");
    if (!std::is_same<T, double>::value && !lds1 && eig2_lds_bytes<T>(nmax) <= LDS_MAX &&
        (sizeof(T) <= 16 || nmax <= 64)) {  // (qd: 8 column slots per lane, n <= 64)
      static std::atomic<unsigned long long> attr2{0}, attr2f{0};
      if (newton) {
        lds_attr_once(attr2, (const void*)eigmin_lds2<T, true>, (int)LDS_MAX);
        eigmin_lds2<T, true><<<(unsigned)h.size(), 512, eig2_lds_bytes<T>(nmax), s>>>(d, out);
      } else {
        lds_attr_once(attr2f, (const void*)eigmin_lds2<T, false>, (int)LDS_MAX);
        eigmin_lds2<T, false><<<(unsigned)h.size(), 512, eig2_lds_bytes<T>(nmax), s>>>(d, out);
      }
      HIPCHK(hipGetLastError());
      return;
    }
    if (eig_lds_bytes<T>(nmax) <= LDS_MAX) {
      const size_t lds = eig_lds_bytes<T>(nmax);
      static std::atomic<unsigned long long> attr_t{0}, attr_f{0};
      lds_attr_once(attr_t, (const void*)eigmin_lds<T, true>, (int)LDS_MAX);
      lds_attr_once(attr_f, (const void*)eigmin_lds<T, false>, (int)LDS_MAX);
      if (newton) eigmin_lds<T, true><<<(unsigned)h.size(), 512, lds, s>>>(d, out);
      else eigmin_lds<T, false><<<(unsigned)h.size(), 512, lds, s>>>(d, out);
    } else {
      const size_t lds = sizeof(T) * (4 * (size_t)nmax + 256);
      eigmin_batched<T><<<(unsigned)h.size(), 256, lds, s>>>(d, out);
    }
    HIPCHK(hipGetLastError());
  }
};


// pivoted LU in place (the approx_lu! / approx_inv! fallback, getrf_batched)
template <class T>
struct LuPlan : PlanBase {
  static constexpr int NB = 16;
  std::vector<LuDesc<T>> h;
  LuDesc<T>* d = nullptr;
  int nmax = 0;
  void add(T* A, int* perm, int n, int lda) {
    h.push_back(LuDesc<T>{A, perm, n, lda});
    nmax = std::max(nmax, n);
  }
  size_t lds = 0;
  // (outside any graph capture: the LDS attribute is set here, not at launch)
  void finalize() {
    if (h.empty()) return;
    d = own(h);
    lds = getrf_lds_bytes<T, NB>(nmax);
    // the static LDS of the kernel (pivot search, pivots) comes on top of the dynamic panel
    if (lds > LDS_MAX - 4096) throw ClrsdpError{CLRSDP_E_ARG, "LU fallback: matrix too large for the on-chip panel"};
    if (lds > 64 * 1024)
      HIPCHK(hipFuncSetAttribute((const void*)getrf_batched<T, NB, 256>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  void launch(hipStream_t s, int* info) const {
    if (h.empty()) return;
    getrf_batched<T, NB, 256><<<(unsigned)h.size(), 256, lds, s>>>(d, info);
    HIPCHK(hipGetLastError());
  }
};

// row gathers out = in[perm, :] (or P I with ident)
template <class T>
struct PermPlan : PlanBase {
  std::vector<PermDesc<T>> h;
  PermDesc<T>* d = nullptr;
  long long emax = 0;
  void add(const T* in, int ldi, T* out, int ldo, const int* perm, int n, int ncol) {
    h.push_back(PermDesc<T>{in, out, perm, n, ncol, ldi, ldo});
    emax = std::max(emax, (long long)n * ncol);
  }
  void finalize() {
    if (!h.empty()) d = own(h);
  }
  void launch(hipStream_t s, bool ident = false) const {
    if (h.empty()) return;
    dim3 g(std::min<unsigned>(cdiv(emax, 256), 64), (unsigned)h.size());
    perm_rows<T><<<g, 256, 0, s>>>(d, ident ? 1 : 0);
    HIPCHK(hipGetLastError());
  }
};

template <class T>
struct CholInvPlan : PlanBase {  // A_b -> L_b^-1 (and optionally L_b)
  std::vector<MatDesc<T>> hin, hout, hl;
  MatDesc<T>*din = nullptr, *dout = nullptr, *dl = nullptr;
  void add(T* A, int n, int lda, T* out, int ldo, T* L = nullptr) {
    hin.push_back(MatDesc<T>{A, n, lda});
    hout.push_back(MatDesc<T>{out, n, ldo});
    nmax = std::max(nmax, n);
    if (L) hl.push_back(MatDesc<T>{L, n, ldo});
  }
  void finalize() {
    if (hin.empty()) return;
    din = own(hin);
    dout = own(hout);
    if (!hl.empty()) dl = own(hl);
  }
  int nmax = 0;
  void launch(hipStream_t s, int* info) const {
    if (hin.empty()) return;
    const unsigned nb = (unsigned)hin.size();
    if constexpr (std::is_same<T, double>::value) {
      if (nmax <= 32) go<32>(s, nb, info);
      else if (nmax <= 64) go<64>(s, nb, info);
      else if (nmax <= 128) go<128>(s, nb, info);
      else go<256>(s, nb, info);
    } else {
      using C = RegCfg<T>;
      static const bool la = !env_off("CLRSDP_CHOL_LA");
      // blocks n <= 32 on 4 waves -- one per SIMD, the chain alone on its SIMD -- instead of 16
      // (C5's X/Y blocks <= 18: 980 -> 1007 it/s, round 5; CLRSDP_LA_SMALL=0 keeps 16)
      static const bool la_small = !env_off("CLRSDP_LA_SMALL");
      if (la && la_small && nmax <= 32) {
        if (std::is_same<T, mw::qd>::value && chol_ldl_on())
          chol_lookahead<T, true, true, 32, 3><<<nb, 256, 0, s>>>(din, dout, dl, info, la_opts());
        else
          chol_lookahead<T, true, false, 32, 3><<<nb, 256, 0, s>>>(din, dout, dl, info, la_opts());
      } else if (la && nmax <= 64) {  // the look-ahead factorisation with L^-1 (SKIP0 as potrf's)
        if (std::is_same<T, mw::qd>::value && chol_ldl_on())
          chol_lookahead<T, true, true, 64, 15, true><<<nb, 1024, 0, s>>>(din, dout, dl, info, la_opts());
        else
          chol_lookahead<T, true, false, 64, 15, true><<<nb, 1024, 0, s>>>(din, dout, dl, info, la_opts());
      } else if (chol_packed_on() && nmax <= 64)
        launch_chol_packed<T, true>(nb, s, din, dout, dl, info);
      else
        chol_inv_reg<T, C::TR, C::TC, C::GR, C::GC><<<nb, C::GR * C::GC, 0, s>>>(din, dout, dl, info);
    }
    HIPCHK(hipGetLastError());
  }
  template <int NP>
  void go(hipStream_t s, unsigned nb, int* info) const {
    // CLRSDP_CHOL_LDS_KB: request at least that much LDS per workgroup, so no 80-KB GEMM
    // workgroup of a side stream can share the CU with a factorisation (A/B experiment)
    static const size_t lds = [] {
      const char* e = std::getenv("CLRSDP_CHOL_LDS_KB");
      const size_t want = e ? (size_t)std::atoi(e) * 1024 : 0;
      return std::min<size_t>(std::max(chol_inv_tiles_lds<NP>(), want), 160 * 1024);
    }();
    // raised wave priority: the factorisation's chains keep their issue slots against the side
    // streams' GEMM waves on the same SIMDs (CLRSDP_CHOL_PRIO=0: default priority)
    static const int prio = env_off("CLRSDP_CHOL_PRIO") ? 0 : 1;
    static std::atomic<unsigned long long> attr{0};
    lds_attr_once(attr, (const void*)chol_inv_tiles<NP>, (int)lds);
    chol_inv_tiles<NP><<<nb, CholTiles<NP>::NTH, lds, s>>>(
        reinterpret_cast<const MatDesc<double>*>(din), reinterpret_cast<const MatDesc<double>*>(dout), info,
        prio);
  }
};

struct HandleBase {
  std::string err;
  int dev = 0;  // the handle's HIP device (every C-ABI call on the handle runs with it current)
  virtual ~HandleBase() {}
  virtual void upload(const double* V, const double* lam, const double* B, const double* c,
                      const double* b, const double* C) = 0;
  virtual void set_state(const double* x, const double* X, const double* y, const double* Y) = 0;
  virtual void get_state(double* x, double* X, double* y, double* Y) = 0;
  virtual int initial(const clrsdp_params* prm, clrsdp_iter_stats* st) = 0;
  virtual int iterate(const clrsdp_params* prm, int pd_feas, clrsdp_iter_stats* st) = 0;
  virtual void set_control(const clrsdp_control* c) = 0;
  virtual int iterate_async(const clrsdp_params* prm) = 0;
  virtual int iterate_wait(clrsdp_iter_stats* st, int* ran) = 0;
  virtual int run_stage(int stage, const clrsdp_params* prm, int pd_feas) = 0;
  virtual void get_buffer(int buf, double* host, int64_t* count) = 0;
  virtual int64_t exchange_bytes() const = 0;
  virtual void set_exchange(clrsdp_exchange_fn fn, void* ctx, void* send, void* recv) = 0;
  virtual void comm_init(const uint8_t* id) = 0;
  virtual void set_stream(void* s) = 0;
  virtual void* get_stream() const = 0;
  virtual void synchronize() = 0;
  virtual void set_timing(int on) = 0;
  virtual void save_state() = 0;
  virtual void restore_state() = 0;
  virtual void set_factorization(int flags) = 0;
  virtual int get_factorization() const = 0;
  virtual void set_graph(int on) = 0;
  virtual void comm_info(int* nranks, int* backend) const = 0;
};

template <class T>
struct Solver final : HandleBase {
  // ---------------- configuration / global description
  int rank = 0, world = 1, timing = 0, W = Num<T>::W;
  int64_t J = 0, n_y = 0;
  std::vector<int64_t> m, Lc, Ns, Ds, xoff_g;    // per cluster
  std::vector<int64_t> jl_first;                 // first (j,l) index of cluster j
  std::vector<int64_t> delta, Kb, nb_g, blkoff_g, voff_g, koff_g;  // per (j,l)
  std::vector<int64_t> rkoff_g;                  // offset into ranks[] of (j,l)
  std::vector<int64_t> ranks_all;
  std::vector<int64_t> Boff_g;                   // per cluster offset in global B
  int64_t tot_x = 0, tot_blk = 0, tot_V = 0, tot_K = 0, tot_B = 0;
  double dimtot = 0;

  // ---------------- local (owned) layout
  std::vector<int> oc;                       // owned clusters (global ids)
  struct LBlk { int c, l; int64_t gjl; int n, del, K, m, N; int64_t off, voff, koff, toff, boff, ayoff, rsoff; };
  std::vector<LBlk> lb;
  std::vector<int64_t> c_xoff, c_Soff, c_Boff;   // per local cluster
  int64_t nx = 0, nblk_el = 0, nV = 0, nK = 0, nT = 0, nBX = 0, nAY = 0, nS = 0, nB = 0, nRS = 0;
  bool anyMgt1 = false, hasC = false;
  bool mw_pair_upper = false;  // BX / BY hold their upper triangles only (schur_assemble reads (min, max))
  int nc2 = 0;  // clusters factorised as 2x2 blocks (s_single < dim_S <= 256, fp64)
  // the largest fp64 S_j factorised (and inverted) by ONE chol_inv_tiles launch: 256 with
  // CLRSDP_CHOL256=1 (chol_inv_tiles<256>, 768 threads: no 2x2 blocking, no X21 / W1 side
  // products), else 128
  const int s_single = (std::is_same<T, double>::value && env_on("CLRSDP_CHOL256")) ? 256 : 128;
  bool s_lower = false;  // the last SCHUR enqueued assembled the lower triangle of S only

  // ---------------- device memory
  hipStream_t own_stream = nullptr, stream = nullptr;
  T *X, *Y, *Xinv, *LX, *LY, *R, *P, *dX, *dY, *Z, *tA, *tB, *Cm;
  T *V, *lam, *TX, *TY, *BX, *BY, *AY, *tval, *S, *Wm, *Bm, *Qslab, *Q, *Qf, *Qinv;
  T *TU, *TW;  // trace_A products U = Z V and the scaled vectors of compute_weighted_A (own
               // buffers: they are produced on the side stream while SCHUR uses TX/TY)
  T *cvec, *x, *dx, *dvec, *rhs, *tvec, *tmpv, *pslab, *y, *bvec, *dyv, *pvec, *uvec;
  T *sc, *bpart, *upart = nullptr, *eigX, *eigY, *tmpsc, *tC = nullptr, *Stmp = nullptr;
  T* Vt = nullptr;  // per block V^T (K x delta), fused Schur path only
  int *ksamp, *rsums, *info;
  T *xsend = nullptr, *xrecv = nullptr, *own_send = nullptr;
  int64_t xcap = 0;  // exchange capacity in T values
  clrsdp_exchange_fn xfn = nullptr;
  void* xctx = nullptr;
  ncclComm_t comm = nullptr;    // native RCCL communicator (clrsdp_comm_init)
  T* comm_recv = nullptr;       // world * xcap values, rank r's partials at r * cnt
  int device = 0;
  bool uploaded = false;
  int info_count = 0, info_S0 = 0, info_Q0 = 0, info_Y0 = 0, info_H = 0;
  int info_L0 = 0;  // status words of X^-1 by LU (one per block)
  int info_G = 0;   // world > 1: the failure bits of every rank, OR-ed (STEP's exchange)
  // ---------------- the LU fallback (approx_lu! / approx_inv!, MPMP.jl:774-786, 1436, 1501):
  // Cholesky first; when a Cholesky status word fires, the loop body is re-run with pivoted LU
  // for S_j and Q (or for X^-1), and LU stays on for the rest of the solve, as the reference
  // switches spd_inv! off.  CLRSDP_FACT_LU_SQ from the start is the reference's own choice.
  int fact_flags = CLRSDP_FACT_FALLBACK;
  bool lu_built = false;
  int* lperm = nullptr;  // row permutations: S_j (at the cluster's x offset), Q, X blocks
  T* W2m = nullptr;      // U_j^-T B_j  (the transposed B_j^T U_j^-1, MPMP.jl:1457-1460)
  bool lu_sq() const { return (fact_flags & CLRSDP_FACT_LU_SQ) != 0; }
  bool lu_x() const { return (fact_flags & CLRSDP_FACT_LU_X) != 0; }
  // pipelined loop (iterate_async / iterate_wait): device-side loop control and results copy
  T gap_thr{}, p_thr{}, d_thr{};
  int need_p = 0, need_d = 0;
  T *Pres = nullptr, *pres = nullptr, *dres = nullptr;  // P, p, d of the last loop body that ran
  bool res_from_copy = false;

  // ---------------- plans
  PlanBase descs;  // owner of the stage descriptor arrays below (d_blk, d_pair, ...)
  GemmPlan<T> p_XY, p_dXdY, p_xinv, p_s1x, p_s1y, p_s2x, p_s2y, p_Q, p_wA_P, p_wA_dX, p_trU_Z,
      p_trU_Y, p_By, p_Btx, p_Wt, p_Wdy, p_PY, p_Z, p_dXY, p_dY;
  TrsmPlan<T> t_Linv, t_W, t_t, t_Q, t_sX1, t_sX2, t_sY1, t_sY2;
  MatPlan<T> f_X, f_Y, f_S, f_Q, e_X, e_Y;
  // on-chip factorisation path (all sizes <= reg_nmax<T>()): L^-1 and MFMA products
  bool reg_blk = false, reg_S = false, reg_Q = false;
  CholInvPlan<T> ci_XY, ci_S, ci_S22, ci_Q;
  GemmPlan<T> q_xinv, q_sx1, q_sx2, q_sy1, q_sy2, q_W, q_t, q_Wdy, q_dx, q_q1, q_q2, q_qinv, q_qdy;
  // fp64, uniform blocks: Z, dY and the step-length products as one strip-chain launch each
  ChainPlan c_Z, c_dY, c_step, c_trZ;
  ChainPlan c_stepX, c_stepY;             // the step-length congruences apart (xy_ov)
  MatPlan<T> e_Xs, e_Ys;                  // their eigen launches apart
  bool xy_ov_ok = false;   // the overlapped step length is configured (small batches, opt-in)
  bool xy_ov_body = false; // enqueue_iteration: the corrector may fork the X step length
  bool xy_ov = false;      // it did: STEP runs the Y half and joins ev_stx
  hipEvent_t ev_dxo = nullptr, ev_stx = nullptr;
  // fp64 FACTOR with every dim_S <= 256 (fac2): f_a = {W = L^-1 B | L21^T = L11^-1 S12, W1} and
  // f_b = {W^T W | S22 - L21 L21^T, W1^T W1, B2 - L21 W1} as mixed batches, then (dim_S > 128)
  // chol_inv(S22), f_c: W2 = L22^-1 B2', f_d: slab += W2^T W2 (measured 1% faster than one
  // W^T W product after W2); f_x1/f_x2: X21 (side stream)
  GemmPlan<T> f_a, f_b, f_c, f_d, f_x1, f_x2;
  // the 2x2-blocked clusters' {W1 = L11^-1 B1} and {W1^T W1, B2 - L21 W1}: off the chain
  // chol(S11) -> L21^T -> S22 - L21 L21^T -> chol(S22'), so a loop body runs them on a second side
  // stream beside it (joined before W2 = L22^-1 B2')
  GemmPlan<T> f_w, f_w2;
  bool fac2 = false;
  T* B2p = nullptr;
  // weighted A with the column scaling inside the GEMM's slab staging (fp64, every local block
  // m = L = 1 with rank-1 samples): no scale_cols launch, no scaled copy of V
  bool wa_fused = false;
  GemmPlan<T> p_wA_Ps, p_wA_dXs;
  // CLRSDP_EXP: development A/B switch for the variant under measurement (0 = the default)
  const int exp_knob = std::getenv("CLRSDP_EXP") ? std::atoi(std::getenv("CLRSDP_EXP")) : 0;
  bool pending_x21 = false;  // the solves wait for X21 (side stream, iterate)
  hipEvent_t ev_x2 = nullptr, ev_x21 = nullptr;
  // multi-word S_j / Q <= 64 in the split form (CLRSDP_MW_SPLIT): potrf on the critical path,
  // L^-1 by four-wave triangular solves of the identity (S_j: on aux2, off the critical path),
  // then the same GEMV solves as the explicit-inverse path
  bool s_split = false, q_split = false, pending_sinv = false;
  bool qf_fresh = false;  // sum_q_slabs wrote Qf = Q for this iteration's factor_q_
  int64_t s_len = 0;
  T *SLi = nullptr, *SLid = nullptr, *QLi = nullptr, *QLid = nullptr;  // L^-1 and identity images
  TrsmPlan<T> t_Sinv, t_Qinv;
  GemmPlan<T> q_t2, q_dx2, q_qinv2;
  hipEvent_t ev_sp = nullptr, ev_sinv = nullptr;
  MatPlan<T> e_XY;                        // both step-length eigenproblems in one launch
  // LU fallback plans (built on the first switch)
  LuPlan<T> lu_S, lu_Q, lu_X;
  PermPlan<T> pm_B, pm_rhs, pm_r, pm_I;
  TrsmPlan<T> tl_W1, tl_W2, tl_t, tl_dx, tl_Q1, tl_Q2, tl_X1, tl_X2;
  GemmPlan<T> lq_slab, lq_Wt;
  BlkDesc* d_blk = nullptr;      // all local blocks
  BlkDesc* d_blk_m = nullptr;    // local blocks with m > 1
  int n_blk_m = 0;
  // fused Schur path (fp64, every local block m = 1): TXt/TYt = V^T X^-1 / V^T Y, then the
  // paired Hadamard tiles; clusters with L > 1 or ranks != 1 are summed from G (BX arena)
  bool fast_schur = false;
  GemmPlan<T> p_txy, p_ty;  // V^T X^-1 (SCHUR) and V^T Y (ahead on the side stream in a loop body)
  bool ty_ahead = false;     // p_ty already enqueued on the side stream (joined by ev_ty)
  hipEvent_t ev_ty = nullptr;
  PairTileDesc* d_ptd = nullptr;
  TileRef* d_pt2d = nullptr;
  int n_ptiles = 0;
  // schur_fused_f64 (every local block delta <= 128): V^T X^-1 formed on chip, one workgroup
  // per 64-row block; CLRSDP_SCHUR_FUSED=0 keeps the V^T X^-1 GEMM + schur_pairs_f64 pair
  bool schur_fused = false;
  bool fused_one = false;   // schur_fused_f64<.., .., .., true>: one column tile per workgroup (small batches)
  bool fused_d64 = false;   // schur_fused_f64<.., .., .., true, true>: the ONE form at delta <= 64
  bool fused_grp2 = false;  // schur_fused_f64<.., .., true>: the rank-2 group-sum epilogue (every block grp = 2)
  bool fused_y = false;  // schur_fused_f64<0, true>: V^T Y on chip too (no p_ty); CLRSDP_SCHUR_FUSED_Y=0
  FusedPairDesc* d_fpd = nullptr;
  TileRef* d_fpt2d = nullptr;
  int n_fwg = 0;
  SchurClusterDesc* d_gcd = nullptr;  // clusters summed by schur_gsum
  int n_gsum = 0, max_gD = 0;
  SchurClusterDesc* d_scd = nullptr;
  SchurBlockDesc* d_sbd = nullptr;
  long long n_pairs = 0;
  AYDesc* d_ayd = nullptr;
  PairDesc* d_pair = nullptr;
  // <X + dX, Y + dY> partials from the predictor's dY chain (dotp, dy_dot_cnt of them)
  T* dotp = nullptr;
  int dy_dot_cnt = 0;
  bool dy_dot_ok = false, dy_dot_ready = false;
  // fp64 cluster solves in two launches (cl_solve_t / cl_solve_dx): one descriptor per cluster,
  // cls_nrb 64-row blocks per cluster (the partial slabs: nc x cls_nrb x n_y in pslab)
  std::vector<ClSolveDesc> h_cls;
  ClSolveDesc* d_cls = nullptr;
  int cls_nrb = 0;
  bool cls_on = false;
  bool trivial_tuples = false;
  int n_pair = 0, max_K = 0;
  ScaleDesc* d_scale = nullptr;
  TupleDesc* d_td = nullptr;
  TupleBlock* d_tb = nullptr;
  hipEvent_t ev[CLRSDP_NUM_STAGES + 1];
  // timing mode 1: inner buckets (CLRSDP_INNER_*), one event pair per segment, recorded on the
  // stream the segment's launches go to (so side-stream work is measured on its own stream)
  std::vector<hipEvent_t> seg_pool;
  std::vector<std::array<int, 3>> segs;  // (bucket, begin event, end event)
  template <class F>
  void seg(int bucket, F&& work) {
    if (timing != 1) {
      work();
      return;
    }
    const int b = (int)segs.size() * 2;
    while ((int)seg_pool.size() < b + 2) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      seg_pool.push_back(e);
    }
    HIPCHK(hipEventRecord(seg_pool[b], stream));
    work();
    HIPCHK(hipEventRecord(seg_pool[b + 1], stream));
    segs.push_back({bucket, b, b + 1});
  }
  // side stream: the local residuals overlap the Schur factorisation, chol(Q) overlaps the
  // first part of the predictor (iterate only; run_stage stays serial)
  hipStream_t aux = nullptr, aux2 = nullptr;
  hipEvent_t ev_m = nullptr, ev_x = nullptr, ev_s = nullptr, ev_r = nullptr, ev_qa = nullptr,
             ev_q = nullptr, ev_join = nullptr, ev_fa = nullptr, ev_w = nullptr, ev_join2 = nullptr;
  bool pending_q = false;
  float phase_ms[CLRSDP_NUM_STAGES];

  int nb() const { return (int)lb.size(); }
  int nc() const { return (int)oc.size(); }

  Solver(const clrsdp_desc* desc, const clrsdp_config* cfg) {
    rank = cfg->rank;
    world = std::max(1, (int)cfg->world_size);
    timing = cfg->timing;
    device = cfg->device;
    dev = cfg->device;
    HIPCHK(hipSetDevice(cfg->device));  // (clrsdp_create restores the caller's device)
    J = desc->J;
    n_y = desc->n_y;
    if (J <= 0 || n_y <= 0) throw ClrsdpError{CLRSDP_E_ARG, "J and n_y must be positive"};
    m.assign(desc->m, desc->m + J);
    Lc.assign(desc->L, desc->L + J);
    Ns.assign(desc->n_samples, desc->n_samples + J);
    int64_t njl = 0;
    for (int64_t j = 0; j < J; ++j) {
      if (m[j] <= 0 || Lc[j] <= 0 || Ns[j] <= 0) throw ClrsdpError{CLRSDP_E_ARG, "bad m/L/N"};
      Ds.push_back(m[j] * (m[j] + 1) / 2 * Ns[j]);
      xoff_g.push_back(tot_x);
      tot_x += Ds[j];
      jl_first.push_back(njl);
      njl += Lc[j];
      Boff_g.push_back(tot_B);
      tot_B += Ds[j] * n_y;
    }
    jl_first.push_back(njl);
    int64_t rk = 0;
    for (int64_t j = 0; j < J; ++j)
      for (int64_t l = 0; l < Lc[j]; ++l) {
        const int64_t g = jl_first[j] + l;
        const int64_t del = desc->delta[g];
        if (del <= 0) throw ClrsdpError{CLRSDP_E_ARG, "bad delta"};
        delta.push_back(del);
        rkoff_g.push_back(rk);
        int64_t K = 0;
        for (int64_t k = 0; k < Ns[j]; ++k) {
          if (desc->ranks[rk + k] < 0) throw ClrsdpError{CLRSDP_E_ARG, "negative rank"};
          K += desc->ranks[rk + k];
          ranks_all.push_back(desc->ranks[rk + k]);
        }
        rk += Ns[j];
        if (K <= 0) throw ClrsdpError{CLRSDP_E_ARG, "block without vectors"};
        Kb.push_back(K);
        const int64_t n = m[j] * del;
        nb_g.push_back(n);
        blkoff_g.push_back(tot_blk);
        tot_blk += n * n;
        voff_g.push_back(tot_V);
        tot_V += del * K;
        koff_g.push_back(tot_K);
        tot_K += K;
        dimtot += (double)n;
      }
    // owned clusters
    if (cfg->owned && cfg->n_owned > 0) {
      for (int i = 0; i < cfg->n_owned; ++i) {
        if (cfg->owned[i] < 0 || cfg->owned[i] >= J) throw ClrsdpError{CLRSDP_E_ARG, "bad owned id"};
        oc.push_back(cfg->owned[i]);
      }
      std::sort(oc.begin(), oc.end());
    } else if (world == 1) {
      for (int j = 0; j < J; ++j) oc.push_back(j);
    }
    // local layout
    for (int c = 0; c < (int)oc.size(); ++c) {
      const int j = oc[c];
      c_xoff.push_back(nx);
      nx += Ds[j];
      c_Soff.push_back(nS);
      nS += Ds[j] * Ds[j];
      c_Boff.push_back(nB);
      nB += Ds[j] * n_y;
      if (std::is_same<T, double>::value && Ds[j] > s_single && Ds[j] <= 256) ++nc2;
      if (m[j] > 1) anyMgt1 = true;
      for (int l = 0; l < Lc[j]; ++l) {
        LBlk b;
        b.c = c; b.l = l; b.gjl = jl_first[j] + l;
        b.n = (int)nb_g[b.gjl]; b.del = (int)delta[b.gjl]; b.K = (int)Kb[b.gjl];
        b.m = (int)m[j]; b.N = (int)Ns[j];
        b.off = nblk_el; nblk_el += (int64_t)b.n * b.n;
        b.voff = nV; nV += (int64_t)b.del * b.K;
        b.koff = nK; nK += b.K;
        b.toff = nT; nT += (int64_t)b.n * b.m * b.K;
        b.boff = nBX; nBX += (int64_t)b.m * b.K * b.m * b.K;
        b.ayoff = nAY; nAY += (int64_t)b.m * (b.m + 1) / 2 * b.K;
        b.rsoff = nRS; nRS += b.N + 1;
        max_K = std::max(max_K, b.K);
        lb.push_back(b);
      }
    }
    fast_schur = std::is_same<T, double>::value && !anyMgt1 && nb() > 0;
    HIPCHK(hipStreamCreateWithFlags(&own_stream, hipStreamNonBlocking));
    stream = own_stream;
    for (auto& e : ev) HIPCHK(hipEventCreate(&e));
    // CLRSDP_ONE_STREAM=1: the side-stream work runs in order on the main stream (experiment:
    // graph-boundary and join idle time against the lost overlap)
    if (env_on("CLRSDP_ONE_STREAM")) {
      aux = aux2 = own_stream;
    } else {
      HIPCHK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
      // CLRSDP_FACTOR_SPLIT=0: FACTOR's W1 products stay on the main stream
      if (env_off("CLRSDP_FACTOR_SPLIT")) aux2 = own_stream;
      else HIPCHK(hipStreamCreateWithFlags(&aux2, hipStreamNonBlocking));
    }
    for (hipEvent_t* e : {&ev_m, &ev_x, &ev_s, &ev_r, &ev_qa, &ev_q, &ev_x2, &ev_x21, &ev_ty, &ev_join,
                          &ev_fa, &ev_w, &ev_join2, &ev_sp, &ev_sinv, &ev_dxo, &ev_stx})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    allocate();
    build_plans();
  }

  ~Solver() override {
    // device memory is released with the process / hipDeviceReset; free what we own explicitly
    T* bufs[] = {X, Y, Xinv, LX, LY, R, P, dX, dY, Z, tA, tB, Cm, V, lam, TX, TY, TU, TW, BX, BY, AY,
                 tval, S, Wm, Bm, Qslab, Q, Qf, Qinv, cvec, x, dx, dvec, rhs, tvec, tmpv, pslab, y,
                 bvec, dyv, pvec, uvec, bpart, upart, eigX, tmpsc, tC, Stmp, B2p, own_send, Vt, Pres, pres, dres,
                 W2m};
    for (T* p : bufs)
      if (p) (void)hipFree(p);
    if (comm) {
      (void)hipStreamSynchronize(stream);
      (void)rccl().comm_destroy(comm);
    }
    if (comm_recv) (void)hipFree(comm_recv);
    if (snap) (void)hipFree(snap);
    if (dotp) (void)hipFree(dotp);
    (void)hipFree(ksamp);
    (void)hipFree(rsums);
    if (lperm) (void)hipFree(lperm);
    if (stat_dev) (void)hipFree(stat_dev);
    if (stat_host) (void)hipHostFree(stat_host);
    for (char* r : ring_host)
      if (r) (void)hipHostFree(r);
    for (auto& e : ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : seg_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ev_m, ev_x, ev_s, ev_r, ev_qa, ev_q, ev_x2, ev_x21, ev_ty, ev_join, ev_fa, ev_w,
                         ev_join2, ev_sp, ev_sinv, ring_ev[0], ring_ev[1]})
      if (e) (void)hipEventDestroy(e);
    for (hipGraphExec_t g : gexec)
      if (g) (void)hipGraphExecDestroy(g);
    if (aux && aux != own_stream) (void)hipStreamDestroy(aux);
    if (aux2 && aux2 != own_stream) (void)hipStreamDestroy(aux2);
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }

  void allocate() {
    const int64_t B = std::max<int64_t>(nblk_el, 1);
    X = dmalloc<T>(B); Y = dmalloc<T>(B); Xinv = dmalloc<T>(B); LX = dmalloc<T>(B);
    LY = dmalloc<T>(B); R = dmalloc<T>(B); P = dmalloc<T>(B); dX = dmalloc<T>(B);
    dY = dmalloc<T>(B); Z = dmalloc<T>(B); tA = dmalloc<T>(B); tB = dmalloc<T>(B);
    Cm = dmalloc<T>(B);
    V = dmalloc<T>(nV); lam = dmalloc<T>(nK);
    // TX / TY: the Schur-stage products; TU / TW (same slot layout, m(m+1)/2 * delta*K <=
    // (m delta)(m K) per block): the trace_A products U and the scaled vectors of
    // compute_weighted_A
    TX = dmalloc<T>(nT); TY = dmalloc<T>(nT); TU = dmalloc<T>(nT); TW = dmalloc<T>(nT);
    BX = dmalloc<T>(nBX); BY = dmalloc<T>(nBX);
    AY = dmalloc<T>(nAY); tval = dmalloc<T>(nAY);
    S = dmalloc<T>(nS); Wm = dmalloc<T>(nB); Bm = dmalloc<T>(nB);
    Qslab = dmalloc<T>((size_t)std::max(nc(), 1) * n_y * n_y);
    Q = dmalloc<T>(n_y * n_y); Qf = dmalloc<T>(n_y * n_y); Qinv = dmalloc<T>(n_y * n_y);
    cvec = dmalloc<T>(nx); x = dmalloc<T>(nx); dx = dmalloc<T>(nx); dvec = dmalloc<T>(nx);
    rhs = dmalloc<T>(nx); tvec = dmalloc<T>(nx); tmpv = dmalloc<T>(nx);
    pslab = dmalloc<T>((size_t)std::max(nc(), 1) * 4 * n_y);  // (x 4: cl_solve_t's row blocks)
    y = dmalloc<T>(n_y); bvec = dmalloc<T>(n_y); dyv = dmalloc<T>(n_y); pvec = dmalloc<T>(n_y);
    Pres = dmalloc<T>(std::max<int64_t>(nblk_el, 1)); pres = dmalloc<T>(std::max<int64_t>(n_y, 1));
    dres = dmalloc<T>(std::max<int64_t>(nx, 1));
    uvec = dmalloc<T>(n_y);
    // sc and the status words share one allocation (one D2H copy per iteration, pinned host
    // mirror) -- see stat_alloc()
    bpart = dmalloc<T>(std::max(nb(), 256));
    upart = dmalloc<T>(3 * RED_G);  // update_state's partial sums
    eigX = dmalloc<T>(2 * std::max(nb(), 1));
    eigY = eigX + std::max(nb(), 1);  // X-side and Y-side minima of one batched eigen launch
    tC = dmalloc<T>(B);
    {
      int64_t ns = 0;
      for (int c = 0; c < nc(); ++c)
        if (std::is_same<T, double>::value && Ds[oc[c]] > s_single && Ds[oc[c]] <= 256) ns += 2 * (Ds[oc[c]] - 128) * 128;
      Stmp = dmalloc<T>(ns);
      int64_t nb2 = 0;
      for (int c = 0; c < nc(); ++c)
        if (std::is_same<T, double>::value && Ds[oc[c]] > s_single && Ds[oc[c]] <= 256) nb2 += (Ds[oc[c]] - 128) * n_y;
      B2p = dmalloc<T>(nb2);
    }
    tmpsc = dmalloc<T>(8);
    ksamp = dmalloc<int>(nK);
    rsums = dmalloc<int>(nRS);
    if (fast_schur) Vt = dmalloc<T>(std::max<int64_t>(nV, 1));
    // info layout: [X: nb][Y: nb][S: nc single + nc2 second blocks][Q: 1][X by LU: nb]
    // [gathered failure bits: 1][halt: 1 (last; not zeroed)]
    info_count = 3 * nb() + nc() + nc2 + 1 + 1 + 1;
    info_H = info_count - 1;
    info_Y0 = nb();
    info_S0 = 2 * nb();
    info_Q0 = 2 * nb() + nc() + nc2;
    info_L0 = info_Q0 + 1;
    info_G = info_L0 + nb();
    stat_alloc();
    xcap = n_y * n_y + n_y + 16;
    own_send = dmalloc<T>(xcap);
    xsend = own_send;
    xrecv = own_send;
    // sample index of every vector column and the rank prefix sums, per local block
    std::vector<int> ks(nK), rs(nRS);
    for (const LBlk& b : lb) {
      const int64_t r0 = rkoff_g[b.gjl];
      int acc = 0, col = 0;
      for (int k = 0; k < b.N; ++k) {
        rs[b.rsoff + k] = acc;
        for (int q = 0; q < ranks_all[r0 + k]; ++q) ks[b.koff + col++] = k;
        acc += (int)ranks_all[r0 + k];
      }
      rs[b.rsoff + b.N] = acc;
    }
    if (nK) HIPCHK(hipMemcpy(ksamp, ks.data(), nK * sizeof(int), hipMemcpyHostToDevice));
    if (nRS) HIPCHK(hipMemcpy(rsums, rs.data(), nRS * sizeof(int), hipMemcpyHostToDevice));
  }

  void build_plans() {
    {
      int nmax_b = 0, nmax_S = 0;
      for (const LBlk& b : lb) nmax_b = std::max(nmax_b, b.n);
      for (int c = 0; c < nc(); ++c) nmax_S = std::max(nmax_S, (int)Ds[oc[c]]);
      reg_blk = nmax_b <= reg_nmax<T>();
      reg_S = nmax_S <= (std::is_same<T, double>::value ? 2 : 1) * reg_nmax<T>();
      reg_Q = n_y <= reg_nmax<T>();
      // multi-word S_j / Q up to 64: GEMV solves with L^-1 instead of the serial multi-word
      // vector solves (four 41-us trsv_wave chains per direction at C5).  Default, the split
      // form: potrf on the critical path and L^-1 = L \ I by four-wave solves (S_j's beside W_j
      // and the Q chain), C5 891 it/s; CLRSDP_MW_SPLIT=0: the look-ahead factorisation with
      // L^-1 (90 us longer per factorisation, 827 it/s; CLRSDP_MW_INV_S=0 / _Q=0 then keep
      // potrf + trsv, 761 it/s).  C4 (dim S_j = 127) unchanged.  Round 5 A/B.
      if (!std::is_same<T, double>::value && !env_off("CLRSDP_CHOL_LA")) {
        static const bool split = !env_off("CLRSDP_MW_SPLIT");
        if (split) {
          // (double-double S_j up to 128: trsv_wave128 forms L^-1 as it does the vector solves)
          const int lim = std::is_same<T, mw::dd>::value && !env_off("CLRSDP_TRSV128") ? 128 : 64;
          s_split = !reg_S && nmax_S <= lim;
          q_split = !reg_Q && n_y <= 64;
        } else {
          if (!env_off("CLRSDP_MW_INV_S")) reg_S = reg_S || nmax_S <= 64;
          if (!env_off("CLRSDP_MW_INV_Q")) reg_Q = reg_Q || n_y <= 64;
        }
      }
    }
    q_xinv.ta = true;
    q_sx2.tb = q_sy2.tb = true;
    // L^-1 dM L^-T exactly symmetric: eigmin_reg reads it without a transposed copy
    q_sx2.sym = std::is_same<T, double>::value;
    f_d.ta = true;
    f_x1.tb = true;
    fac2 = std::is_same<T, double>::value && reg_S;
    q_dx.ta = true;
    q_q2.ta = true;
    p_xinv.ta = true;
    p_s2x.ta = p_s2y.ta = true;
    // (multi-word, every block m = 1: only the upper tiles of the symmetric pairings; CLRSDP_MW_PAIR_UPPER=0
    // computes both triangles)
    mw_pair_upper = !std::is_same<T, double>::value && !anyMgt1 && !env_off("CLRSDP_MW_PAIR_UPPER");
    p_s2x.upper = p_s2y.upper = mw_pair_upper;
    p_Q.ta = true;
    p_wA_P.tb = p_wA_dX.tb = true;
    p_Btx.ta = true;
    p_Wt.ta = true;
    std::vector<BlkDesc> bd, bdm;
    std::vector<AYDesc> ayd;
    std::vector<PairDesc> pd;
    std::vector<ScaleDesc> sd;
    for (const LBlk& b : lb) {
      const int n = b.n, del = b.del, K = b.K, mm = b.m;
      BlkDesc d{b.off, n, 0};
      bd.push_back(d);
      if (mm > 1) bdm.push_back(d);
      p_XY.add(X + b.off, n, Y + b.off, n, nullptr, n, R + b.off, n, n, n, n);
      p_dXdY.add(dX + b.off, n, dY + b.off, n, R + b.off, n, R + b.off, n, n, n, n);
      p_xinv.add(tA + b.off, n, tA + b.off, n, nullptr, n, Xinv + b.off, n, n, n, n);
      p_PY.add(P + b.off, n, Y + b.off, n, R + b.off, n, tA + b.off, n, n, n, n);
      p_Z.add(Xinv + b.off, n, tA + b.off, n, nullptr, n, Z + b.off, n, n, n, n);
      p_dXY.add(dX + b.off, n, Y + b.off, n, R + b.off, n, tA + b.off, n, n, n, n);
      p_dY.add(Xinv + b.off, n, tA + b.off, n, nullptr, n, dY + b.off, n, n, n, n);
      t_Linv.add(LX + b.off, n, tA + b.off, n, n, n);
      t_sX1.add(LX + b.off, n, tA + b.off, n, n, n);
      t_sX2.add(LX + b.off, n, tB + b.off, n, n, n);
      t_sY1.add(LY + b.off, n, tA + b.off, n, n, n);
      t_sY2.add(LY + b.off, n, tB + b.off, n, n, n);
      f_X.add(LX + b.off, n, n);
      f_Y.add(LY + b.off, n, n);
      ci_XY.add(X + b.off, n, n, LX + b.off, n);
      q_xinv.add(LX + b.off, n, LX + b.off, n, nullptr, n, Xinv + b.off, n, n, n, n);
      if constexpr (std::is_same<T, double>::value) {
        p_xir.add_op(true, false, 1.0, 0.0, LX + b.off, n, LX + b.off, n, nullptr, n, Xinv + b.off, n, n, n, n);
        p_xir.add_op(false, false, -1.0, 0.0, X + b.off, n, Y + b.off, n, nullptr, n, R + b.off, n, n, n, n);
        if (!p_xir.h.empty()) {
          p_xir.h.back().flags |= 16;  // + mu_p I
          p_xir.h.back().sa = sc + SC_MU_P;
        }
      }
      // step length: L^-1 dM L^-T for X and Y in the same two launches (Y's middle product in Z)
      q_sx1.add(LX + b.off, n, dX + b.off, n, nullptr, n, tA + b.off, n, n, n, n);
      q_sx1.add(LY + b.off, n, dY + b.off, n, nullptr, n, Z + b.off, n, n, n, n);
      q_sx2.add(tA + b.off, n, LX + b.off, n, nullptr, n, tB + b.off, n, n, n, n);
      q_sx2.add(Z + b.off, n, LY + b.off, n, nullptr, n, tC + b.off, n, n, n, n);
      e_X.add(tB + b.off, n, n);
      e_Y.add(tB + b.off, n, n);
      e_XY.add(tB + b.off, n, n);
      const int ldT = n;           // TX_b is (m delta) x (m K)
      const int ldBX = mm * K;     // BX_b is (m K) x (m K)
      for (int s = 0; s < mm; ++s) {
        p_s1x.add(Xinv + b.off + (int64_t)s * del * n, n, V + b.voff, del, nullptr, 0,
                  TX + b.toff + (int64_t)s * K * ldT, ldT, n, K, del);
        p_s1y.add(Y + b.off + (int64_t)s * del * n, n, V + b.voff, del, nullptr, 0,
                  TY + b.toff + (int64_t)s * K * ldT, ldT, n, K, del);
        for (int r = 0; r < mm; ++r) {
          p_s2x.add(V + b.voff, del, TX + b.toff + r * del + (int64_t)s * K * ldT, ldT, nullptr, 0,
                    BX + b.boff + r * K + (int64_t)s * K * ldBX, ldBX, K, K, del);
          p_s2y.add(V + b.voff, del, TY + b.toff + r * del + (int64_t)s * K * ldT, ldT, nullptr, 0,
                    BY + b.boff + r * K + (int64_t)s * K * ldBX, ldBX, K, K, del);
        }
      }
      ayd.push_back(AYDesc{b.boff, b.ayoff, K, mm});
      const int64_t xo = c_xoff[b.c];
      for (int r = 0; r < mm; ++r)
        for (int s = 0; s <= r; ++s) {
          const int rsi = s + r * (r + 1) / 2;
          const int64_t uoff = b.toff + (int64_t)rsi * del * K;  // U / Vs slot in TU / TW
          // trace_A: U = Z[r,s] V   (Z block rows r, cols s)
          p_trU_Z.add(Z + b.off + r * del + (int64_t)s * del * n, n, V + b.voff, del, nullptr, 0,
                      TU + uoff, del, del, K, del);
          p_trU_Y.add(Y + b.off + r * del + (int64_t)s * del * n, n, V + b.voff, del, nullptr, 0,
                      TU + uoff, del, del, K, del);
          pd.push_back(PairDesc{uoff, b.voff, b.ayoff + (int64_t)rsi * K, del, K, (int)b.koff,
                                -1});
          // weighted A: block (s, r) = Vs V^T  (MPMP.jl:1659-1667)
          ScaleDesc s_;
          s_.v_off = b.voff; s_.vs_off = uoff; s_.delta = del; s_.K = K;
          s_.ks_off = (int)b.koff; s_.lam_off = (int)b.koff;
          s_.a_off = (int)(xo + (int64_t)rsi * b.N);
          s_.scale = (r != s) ? 0.5 : 1.0;
          sd.push_back(s_);
          // P = WA(x) - X and dX = WA(dx) + P: the second term rides in the GEMM's Cin
          const int64_t so = s * del + (int64_t)r * del * n;
          p_wA_P.add(TW + uoff, del, V + b.voff, del, X + b.off + so, n, P + b.off + so, n, del,
                     del, K);
          p_wA_dX.add(TW + uoff, del, V + b.voff, del, P + b.off + so, n, dX + b.off + so, n,
                      del, del, K);
        }
    }
    for (const LBlk& b : lb) ci_XY.add(Y + b.off, b.n, b.n, LY + b.off, b.n);
    for (const LBlk& b : lb) e_XY.add(tC + b.off, b.n, b.n);
    if constexpr (std::is_same<T, double>::value) {
      // the strip chains need one block size n <= 128 at stride n^2 (one cluster shape: C3 and
      // its shards); by default taken for 64 < n (C2's n = 64 keeps the tiled GEMMs); Z only for
      // m = 1 (no symmetrisation of Z); CLRSDP_CHAIN=0 / 1 forces either
      const char* ec = std::getenv("CLRSDP_CHAIN");
      bool uni_blk = !lb.empty() && !anyMgt1;
      for (size_t q = 0; q < lb.size() && uni_blk; ++q)
        uni_blk = lb[q].n == lb[0].n && lb[q].off == lb[0].off + (int64_t)q * lb[0].n * lb[0].n;
      const int n0 = lb.empty() ? 0 : lb[0].n;
      const bool chains = uni_blk && n0 <= 128 && reg_blk && !(ec && ec[0] == '0') &&
                          ((ec && ec[0] == '1') || n0 > 64);
      if (chains) {
        const int nbk = (int)lb.size();
        c_Z.init(n0, nbk, 1, false, false);
        c_Z.set(0, P, Y, R, Xinv, Z);            // Z = X^-1 (P Y - R)
        c_dY.init(n0, nbk, 1, false, false);
        c_dY.set(0, dX, Y, R, Xinv, dY);         // dY = X^-1 (R - dX Y)
        // the predictor's dY launch also leaves the partials of <X + dX, Y + dY> (CORRECTOR_R's
        // mu; a flat sum over both triangles, so dY before its symmetrisation gives the same
        // value); one rank only (CLRSDP_DY_DOT=0: the separate flat_reduce)
        static const bool dd_env = !env_off("CLRSDP_DY_DOT");
        dy_dot_cnt = nbk * (int)cdiv(n0, chain::NS);
        dy_dot_ok = dd_env && world == 1;
        if (dy_dot_ok) {
          if (!dotp) dotp = dmalloc<T>(dy_dot_cnt);
          c_dY.u.DA[0] = X; c_dY.u.DdA[0] = dX; c_dY.u.DB[0] = Y;
        }
        c_step.init(n0, nbk, 2, true, true);
        c_step.set(0, dX, LX, nullptr, LX, tB);  // L_X^-1 dX L_X^-T
        c_step.set(1, dY, LY, nullptr, LY, tC);  // L_Y^-1 dY L_Y^-T
        // the X and Y halves apart, for the overlapped step length of small batches (below)
        c_stepX.init(n0, nbk, 1, true, true);
        c_stepX.set(0, dX, LX, nullptr, LX, tB);
        c_stepY.init(n0, nbk, 1, true, true);
        c_stepY.set(0, dY, LY, nullptr, LY, tC);
        for (const LBlk& b : lb) {
          e_Xs.add(tB + b.off, b.n, b.n);
          e_Ys.add(tC + b.off, b.n, b.n);
        }
        e_Xs.finalize();
        e_Ys.finalize();
        // CLRSDP_XY_OVERLAP=1 (round 6): with at most
        // CLRSDP_XY_OVERLAP_MAX (32) local blocks the X step length (its congruence and eigen
        // launch) runs on the side stream as soon as the corrector's dX exists, beside dY and
        // the Y step length.  Measured, not the default.
        const char* eo = std::getenv("CLRSDP_XY_OVERLAP_MAX");
        xy_ov_ok = env_on("CLRSDP_XY_OVERLAP") && nb() <= (eo ? std::atoi(eo) : 32);
      }
    }
    n_blk_m = (int)bdm.size();
    if (std::is_same<T, double>::value && !env_off("CLRSDP_SYM_TILES")) {
      int nmx = 0;
      for (const LBlk& b : lb) nmx = std::max(nmx, b.n);
      const int nt = (nmx + 31) / 32;
      sym_pairs = nt * (nt + 1) / 2;
    }
    d_blk = descs.own(bd);
    if (n_blk_m) d_blk_m = descs.own(bdm);
    d_ayd = descs.own(ayd);
    build_ozaki();
    n_pair = (int)pd.size();
    // tuples <-> columns 1:1 in every local cluster (m = L = 1, every rank 1): fused trace_A
    trivial_tuples = n_pair > 0;
    {
      int bi = 0, pi = 0;
      for (int c = 0; c < nc() && trivial_tuples; ++c) {
        const int j = oc[c];
        trivial_tuples = m[j] == 1 && Lc[j] == 1;
        for (int k = 0; k < Ns[j] && trivial_tuples; ++k)
          trivial_tuples = ranks_all[rkoff_g[lb[bi].gjl] + k] == 1;
        if (trivial_tuples) pd[pi].x_off = (int)c_xoff[c];
        bi += (int)Lc[j];
        pi += 1;
      }
    }
    d_pair = descs.own(pd);
    d_scale = descs.own(sd);
    // U = Z V and the column sums of the right-hand side in one launch (chain_f64 TRACE): with
    // the Z chain, trivial tuples and every block's K, lambda and tuple slices at fixed strides
    if constexpr (std::is_same<T, double>::value) {
      bool tr = c_Z.on && trivial_tuples && (int)pd.size() == (int)lb.size();
      for (size_t q = 0; q < pd.size() && tr; ++q)
        tr = pd[q].K == pd[0].K && pd[q].delta == lb[0].n && pd[q].v_off == pd[0].v_off + (long long)q * pd[0].delta * pd[0].K &&
             (long long)pd[q].lam_off == pd[0].lam_off + (long long)q * pd[0].K &&
             (long long)pd[q].x_off == pd[0].x_off + (long long)q * pd[0].K;
      if (tr) {
        c_trZ.init(lb[0].n, (int)lb.size(), 1, false, false);
        c_trZ.trace = true;
        c_trZ.set(0, Z, V + pd[0].v_off, nullptr, nullptr, nullptr);
        c_trZ.u.ldb1 = pd[0].delta;
        c_trZ.u.sB1 = (long long)pd[0].delta * pd[0].K;
        c_trZ.u.NC = pd[0].K;
        c_trZ.u.lam = lam + pd[0].lam_off;
        c_trZ.u.sLam = pd[0].K;
        c_trZ.u.din = dvec + pd[0].x_off;
        c_trZ.u.rout = rhs + pd[0].x_off;
        c_trZ.u.sX = pd[0].K;
        c_trZ.u.c_in = -1.0;  // rhs_x = -d - Tr(A_* Z)  (MPMP.jl:1733-1739)
        c_trZ.u.c_agg = -1.0;
      }
    }
    // trivial tuples + fp64 + the fused Schur layout: x_i / dx_i of column p is entry p of the
    // cluster's slice, lambda_p entry p of the block's
    wa_fused = std::is_same<T, double>::value && trivial_tuples && fast_schur;
    if (wa_fused) {
      p_wA_Ps.tb = p_wA_dXs.tb = true;
      for (const LBlk& b : lb) {
        const int n = b.n, del = b.del, K = b.K;
        const int64_t xo = c_xoff[b.c];
        p_wA_Ps.add_scaled(V + b.voff, del, V + b.voff, del, X + b.off, n, P + b.off, n, del, del, K,
                           x + xo, lam + b.koff);
        p_wA_dXs.add_scaled(V + b.voff, del, V + b.voff, del, P + b.off, n, dX + b.off, n, del, del, K,
                            dx + xo, lam + b.koff);
      }
    }
    // per cluster plans
    std::vector<SchurClusterDesc> scd;
    std::vector<SchurBlockDesc> sbd;
    h_cls.clear();
    cls_nrb = 0;
    cls_on = false;
    std::vector<TupleDesc> td;
    std::vector<TupleBlock> tbk;
    int bi = 0;
    int64_t s2off = 0, b2off = 0;
    std::vector<MatDesc<T>> s11;  // S11 blocks of the 2x2-blocked clusters (chol_inv in ci_S)
    if (s_split || q_split) {
      q_dx2.ta = true;
      q_qinv2.ta = true;
      t_W.four = t_Sinv.four = t_Qinv.four = true;
      auto ident = [&](T*& img, T*& id, const std::vector<std::pair<int64_t, int>>& blocks, int64_t len) {
        img = dmalloc<T>(len);
        id = dmalloc<T>(len);
        std::vector<T> h((size_t)len, T(0.0));
        for (const auto& b : blocks)
          for (int i = 0; i < b.second; ++i) h[(size_t)(b.first + (int64_t)i * b.second + i)] = T(1.0);
        HIPCHK(hipMemcpy(id, h.data(), (size_t)len * sizeof(T), hipMemcpyHostToDevice));
      };
      if (s_split) {
        std::vector<std::pair<int64_t, int>> bl;
        int64_t len = 1;
        for (int c = 0; c < nc(); ++c) {
          const int D = (int)Ds[oc[c]];
          bl.push_back({c_Soff[c], D});
          len = std::max(len, c_Soff[c] + (int64_t)D * D);
        }
        ident(SLi, SLid, bl, len);
        s_len = len;
      }
      if (q_split) ident(QLi, QLid, {{0, (int)n_y}}, std::max<int64_t>(n_y * n_y, 1));
    }
    for (int c = 0; c < nc(); ++c) {
      const int j = oc[c];
      const int D = (int)Ds[j];
      T* Sc = S + c_Soff[c];
      T* Wc = Wm + c_Boff[c];
      T* Bc = Bm + c_Boff[c];
      const int64_t xo = c_xoff[c];
      f_S.add(Sc, D, D);
      T* slab = Qslab + (int64_t)c * n_y * n_y;
      const int ny = (int)n_y;
      if (!std::is_same<T, double>::value || D <= s_single) {
        ci_S.add(Sc, D, D, Sc, D);
        q_W.add(Sc, D, Bc, D, nullptr, 0, Wc, D, D, ny, D);
        if (std::is_same<T, double>::value) {  // (mixed batches are fp64 only)
          f_a.add_op(false, false, 1.0, 0.0, Sc, D, Bc, D, nullptr, 0, Wc, D, D, ny, D);    // W = L^-1 B
          f_b.add_op(true, false, 1.0, 0.0, Wc, D, Wc, D, nullptr, 0, slab, ny, ny, ny, D); // W^T W
        }
        q_t.add(Sc, D, rhs + xo, D, nullptr, 0, tvec + xo, D, D, 1, D);
        q_dx.add(Sc, D, tmpv + xo, D, nullptr, 0, dx + xo, D, D, 1, D);
      } else if (D <= 256) {
        // S = [S11 S12; S21 S22] = L L^T with L = [L11 0; L21 L22] (SURVEY.md §3D with Cholesky):
        // the critical path only needs W = L^-1 B and Q's slab; X21 = -L22^-1 L21 L11^-1 (the
        // lower-left block of L^-1, for the solves) is formed on the side stream
        const int D1 = 128, D2 = D - 128;
        T* S11 = Sc;
        T* S12 = Sc + (int64_t)D1 * D;
        T* S21 = Sc + D1;
        T* S22 = Sc + D1 + (int64_t)D1 * D;
        T* T12 = Stmp + s2off;               // L11^-1 S12 = L21^T   (D1 x D2)
        T* Mb = T12 + (int64_t)D2 * D1;      // L22^-1 L21           (D2 x D1)
        T* B2 = B2p + b2off;                 // B2 - L21 W1          (D2 x n_y)
        s2off += 2 * (int64_t)D2 * D1;
        b2off += (int64_t)D2 * n_y;
        s11.push_back(MatDesc<T>{S11, D1, D});                                          // S11 <- L11^-1
        // (S21^T, not S12: the fused Schur kernel may assemble only the lower triangle)
        f_a.add_op(false, true, 1.0, 0.0, S11, D, S21, D, nullptr, 0, T12, D1, D1, D2, D1);
        f_w.add_op(false, false, 1.0, 0.0, S11, D, Bc, D, nullptr, 0, Wc, D, D1, ny, D1);  // W1
        f_b.add_op(true, false, -1.0, 1.0, T12, D1, T12, D1, S22, D, S22, D, D2, D2, D1);  // S22 - L21 L21^T
        f_w2.add_op(true, false, 1.0, 0.0, Wc, D, Wc, D, nullptr, 0, slab, ny, ny, ny, D1); // W1^T W1
        f_w2.add_op(true, false, -1.0, 1.0, T12, D1, Wc, D, Bc + D1, D, B2, D2, D2, ny, D1);  // B2'
        ci_S22.add(S22, D2, D, S22, D);                                                 // S22 <- L22^-1
        f_c.add(S22, D, B2, D2, nullptr, 0, Wc + D1, D, D2, ny, D2);                   // W2 = L22^-1 B2'
        f_d.add(Wc + D1, D, Wc + D1, D, slab, ny, slab, ny, ny, ny, D2);               // slab += W2^T W2
        f_x1.add(S22, D, T12, D1, nullptr, 0, Mb, D2, D2, D1, D2);                      // M = L22^-1 L21
        f_x2.add(Mb, D2, S11, D, nullptr, 0, S21, D, D2, D1, D1);                       // S21 <- -M L11^-1
        // S12 is not part of L^-1: the products with L^-1 below are split so that none reads it
        q_t.add(S11, D, rhs + xo, D, nullptr, 0, tvec + xo, D, D1, 1, D1);
        q_t.add(Sc + D1, D, rhs + xo, D, nullptr, 0, tvec + xo + D1, D, D2, 1, D);
        // dx = (L^-1)^T u: columns 0..D1-1 of L^-1 are [L11^-1; X21], the rest L22^-1
        q_dx.add(Sc, D, tmpv + xo, D, nullptr, 0, dx + xo, D, D1, 1, D);
        q_dx.add(S22, D, tmpv + xo + D1, D2, nullptr, 0, dx + xo + D1, D2, D2, 1, D2);
      } else {
        q_t.add(Sc, D, rhs + xo, D, nullptr, 0, tvec + xo, D, D, 1, D);
        q_dx.add(Sc, D, tmpv + xo, D, nullptr, 0, dx + xo, D, D, 1, D);
      }
      q_Wdy.add(Wc, D, dyv, (int)n_y, tvec + xo, D, tmpv + xo, D, D, 1, (int)n_y);
      t_W.add(Sc, D, Wc, D, D, (int)n_y, false, Bc);
      t_t.add(Sc, D, tvec + xo, D, D, 1);
      if (s_split) {
        T* Li = SLi + c_Soff[c];
        t_Sinv.add(Sc, D, Li, D, D, D, true);                                        // L^-1 = L \ I
        q_t2.add(Li, D, rhs + xo, D, nullptr, 0, tvec + xo, D, D, 1, D);
        q_dx2.add(Li, D, tmpv + xo, D, nullptr, 0, dx + xo, D, D, 1, D);
      }
      p_Q.add(Wc, D, Wc, D, nullptr, 0, slab, ny, ny, ny, D);
      p_By.add(Bc, D, y, (int)n_y, nullptr, 0, tmpv + xo, D, D, 1, (int)n_y);
      p_Btx.add(Bc, D, x + xo, D, nullptr, 0, pslab + (int64_t)c * n_y, (int)n_y, (int)n_y, 1, D);
      p_Wt.add(Wc, D, tvec + xo, D, nullptr, 0, pslab + (int64_t)c * n_y, (int)n_y, (int)n_y, 1, D);
      p_Wdy.add(Wc, D, dyv, (int)n_y, tvec + xo, D, dx + xo, D, D, 1, (int)n_y);
      if constexpr (std::is_same<T, double>::value) {
        ClSolveDesc cs{};
        cs.L = Sc; cs.W = Wc; cs.rhs = rhs + xo; cs.t = tvec + xo; cs.dx = dx + xo; cs.D = D;
        h_cls.push_back(cs);
        cls_nrb = std::max(cls_nrb, (int)cdiv(D, 64));
      }
      SchurClusterDesc cdsc;
      cdsc.m = (int)m[j]; cdsc.N = (int)Ns[j]; cdsc.D = D;
      cdsc.blk0 = bi; cdsc.nblk = (int)Lc[j];
      cdsc.pair0 = (int)n_pairs;
      cdsc.S_off = c_Soff[c];
      scd.push_back(cdsc);
      n_pairs += (long long)D * (D + 1) / 2;
      TupleDesc tdc;
      tdc.x_off = (int)xo; tdc.N = (int)Ns[j]; tdc.m = (int)m[j];
      tdc.blk0 = bi; tdc.nblk = (int)Lc[j]; tdc.t0 = (int)xo;
      td.push_back(tdc);
      for (int l = 0; l < Lc[j]; ++l, ++bi) {
        const LBlk& b = lb[bi];
        SchurBlockDesc s;
        s.bx_off = b.boff; s.K = b.K; s.rs_off = (int)b.rsoff; s.lam_off = (int)b.koff; s.pad = 0;
        sbd.push_back(s);
        TupleBlock t;
        t.val_off = b.ayoff; t.K = b.K; t.rs_off = (int)b.rsoff; t.lam_off = (int)b.koff; t.pad = 0;
        tbk.push_back(t);
      }
    }
    for (const MatDesc<T>& m1 : s11) ci_S.add(m1.A, m1.n, m1.lda, m1.A, m1.lda);  // after the single blocks
    t_Q.add(Qf, (int)n_y, dyv, (int)n_y, (int)n_y, 1);
    t_dxadd_init();
    f_Q.add(Qf, (int)n_y, (int)n_y);
    ci_Q.add(Q, (int)n_y, (int)n_y, Qf, (int)n_y);
    q_q1.add(Qf, (int)n_y, dyv, (int)n_y, nullptr, 0, uvec, (int)n_y, (int)n_y, 1, (int)n_y);
    q_q2.add(Qf, (int)n_y, uvec, (int)n_y, nullptr, 0, dyv, (int)n_y, (int)n_y, 1, (int)n_y);
    // Q^-1 = L_Q^-T L_Q^-1 once per iteration (side stream), then one GEMV per direction
    q_qinv.ta = true;
    q_qinv.add(Qf, (int)n_y, Qf, (int)n_y, nullptr, 0, Qinv, (int)n_y, (int)n_y, (int)n_y, (int)n_y);
    q_qdy.add(Qinv, (int)n_y, uvec, (int)n_y, nullptr, 0, dyv, (int)n_y, (int)n_y, 1, (int)n_y);
    if (q_split) {
      t_Qinv.add(Qf, (int)n_y, QLi, (int)n_y, (int)n_y, (int)n_y, true);            // L_Q^-1 = L_Q \ I
      q_qinv2.add(QLi, (int)n_y, QLi, (int)n_y, nullptr, 0, Qinv, (int)n_y, (int)n_y, (int)n_y, (int)n_y);
    }
    {
      // (fp64 explicit inverses of S_j (<= 256) and Q; opt-in, CLRSDP_CL_SOLVE=1: at C3 the two
      // launches ran 14.8 + 21.4 us against 13.4 + 11.8 for the four GEMVs, and slab_qsolve
      // summing four partial slabs per cluster 13.7 against 9.0 us: 1195-1232 against 1248-1270
      // it/s, A/B round 5 -- fewer workgroups with longer load chains lose to more, shorter ones)
      const bool cl_env = env_on("CLRSDP_CL_SOLVE");  // (per handle: tests switch it)
      const long long cnt = (long long)std::max(nc(), 1) * std::max(cls_nrb, 1);
      cls_on = cl_env && std::is_same<T, double>::value && reg_S && reg_Q && nc() > 0 &&
               cls_nrb <= 4 && (long long)cdiv(n_y, 64) * cnt * n_y <= (1LL << 20) &&
               ((size_t)n_y + 256) * sizeof(double) <= 64 * 1024;
      for (const ClSolveDesc& cs : h_cls) cls_on = cls_on && cs.D <= 256;
      if (cls_on) d_cls = descs.own(h_cls);
    }
    if (nc()) {
      d_scd = descs.own(scd);
      d_sbd = descs.own(sbd);
      d_td = descs.own(td);
      d_tb = descs.own(tbk);
    }
    if (fast_schur) build_fast_schur();
    {  // FACTOR's critical-path products run beside the side streams' P, Z and W1 work: raised
       // wave priority, opt-in with CLRSDP_FACTOR_PRIO=1 (C3 1252-1276 against 1260-1266 it/s,
       // A/B round 5: the contention is for CUs, not for issue slots)
      static const bool fp = env_on("CLRSDP_FACTOR_PRIO");
      f_a.prio = f_b.prio = f_c.prio = f_d.prio = fp;
    }
    for (GemmPlan<T>* g : {&p_txy, &p_ty, &p_XY, &p_dXdY, &p_xinv, &p_s1x, &p_s1y, &p_s2x, &p_s2y, &p_Q, &p_wA_P,
                           &p_wA_dX, &p_trU_Z, &p_trU_Y, &p_By, &p_Btx, &p_Wt, &p_Wdy, &p_PY,
                           &p_Z, &p_dXY, &p_dY, &q_xinv, &q_sx1, &q_sx2, &q_sy1, &q_sy2, &q_W,
                           &q_t, &q_Wdy, &q_dx, &q_q1, &q_q2, &q_qinv, &q_qdy, &f_a, &f_b, &f_c, &f_d, &f_x1, &f_x2, &f_w, &f_w2,
                           &q_t2, &q_dx2, &q_qinv2,
                           &p_wA_Ps, &p_wA_dXs, &p_xir})
      g->finalize();
    for (CholInvPlan<T>* c : {&ci_XY, &ci_S, &ci_S22, &ci_Q}) c->finalize();
    e_XY.finalize();
    for (TrsmPlan<T>* t : {&t_Linv, &t_W, &t_t, &t_Q, &t_sX1, &t_sX2, &t_sY1, &t_sY2, &t_dx, &t_Sinv, &t_Qinv})
      t->finalize();
    for (MatPlan<T>* f : {&f_X, &f_Y, &f_S, &f_Q}) f->reg_potrf = true;
    for (MatPlan<T>* f : {&f_X, &f_Y, &f_S, &f_Q, &e_X, &e_Y}) f->finalize();
  }

  // ---- double-double Schur products on the int8 matrix cores (Ozaki scheme, oz_split / oz_gemm in
  // kernels_dense.h; round 6): every block m = 1.  Four launches replace the four gemm_valu_ks
  // launches of p_s1x, p_s1y, p_s2x, p_s2y: the digits of the rows of X^-1_b and Y_b and of the
  // columns of V_b; TX_b = X^-1_b V_b and TY_b = Y_b V_b; the digits of the columns of TX_b, TY_b;
  // BX_b = V_b^T TX_b and BY_b = V_b^T TY_b on their upper 16-tiles (the rows of V_b^T are the
  // columns of V_b, so their digits serve twice).  CLRSDP_OZAKI=0 keeps the VALU products.
  bool use_oz = false;
  OzSplitDesc* d_ozs1 = nullptr;
  OzSplitDesc* d_ozs2 = nullptr;
  OzGemmDesc* d_ozg1 = nullptr;
  OzGemmDesc* d_ozg2 = nullptr;
  TileRef *d_ozs1t = nullptr, *d_ozs2t = nullptr, *d_ozg1t = nullptr, *d_ozg2t = nullptr;
  int n_ozs1 = 0, n_ozs2 = 0, n_ozg1 = 0, n_ozg2 = 0;
  void build_ozaki() {
    use_oz = false;
    if constexpr (std::is_same<T, mw::dd>::value) {
      if (anyMgt1 || lb.empty() || env_off("CLRSDP_OZAKI")) return;
      std::vector<OzSplitDesc> s1, s2;
      std::vector<OzGemmDesc> g1, g2;
      std::vector<TileRef> s1t, s2t, g1t, g2t;
      auto pad = [](int v, int q) { return (v + q - 1) / q * q; };
      auto digits = [&](int nv, int K) {
        signed char* D = dmalloc<signed char>((size_t)OZ_S * pad(nv, 16) * pad(K, 64));
        descs.owned_dev.push_back(D);
        return D;
      };
      auto expo = [&](int nv) {
        int* E = dmalloc<int>((size_t)pad(nv, 16));
        descs.owned_dev.push_back(E);
        return E;
      };
      auto add_split = [&](std::vector<OzSplitDesc>& v, std::vector<TileRef>& t, const T* X, long long sv,
                           long long sk, int nv, int K, signed char* D, int* E) {
        v.push_back(OzSplitDesc{X, sv, sk, D, E, nv, K, pad(nv, 16), pad(K, 64)});
        for (int g = 0; g < cdiv(nv, 4); ++g) t.push_back(TileRef{(int)v.size() - 1, g});
      };
      auto add_gemm = [&](std::vector<OzGemmDesc>& v, std::vector<TileRef>& t, const signed char* DA,
                          const int* EA, int RA, const signed char* DB, const int* EB, int RB, int Kp,
                          T* C, int ldc, int M, int N, bool upper) {
        const int tn = cdiv(N, 16);
        v.push_back(OzGemmDesc{DA, EA, DB, EB, C, RA, RB, Kp, ldc, M, N, tn, 0});
        for (int q = 0; q < cdiv(M, 16) * tn; ++q)
          if (!upper || q / tn <= q % tn) t.push_back(TileRef{(int)v.size() - 1, q});
      };
      for (const LBlk& b : lb) {
        const int n = b.n, del = b.del, K = b.K;
        if (K <= 0 || del <= 0) continue;
        signed char *Dx = digits(n, del), *Dy = digits(n, del), *Gv = digits(K, del);
        signed char *Gtx = digits(K, del), *Gty = digits(K, del);
        int *Ex = expo(n), *Ey = expo(n), *Fv = expo(K), *Ftx = expo(K), *Fty = expo(K);
        // rows of X^-1_b, Y_b (n x n, ld n: row v, element k at v + k n); columns of V_b (del x K)
        add_split(s1, s1t, Xinv + b.off, 1, n, n, del, Dx, Ex);
        add_split(s1, s1t, Y + b.off, 1, n, n, del, Dy, Ey);
        add_split(s1, s1t, V + b.voff, del, 1, K, del, Gv, Fv);
        // columns of TX_b, TY_b (del x K, ld n)
        add_split(s2, s2t, TX + b.toff, n, 1, K, del, Gtx, Ftx);
        add_split(s2, s2t, TY + b.toff, n, 1, K, del, Gty, Fty);
        const int Kp = pad(del, 64);
        add_gemm(g1, g1t, Dx, Ex, pad(n, 16), Gv, Fv, pad(K, 16), Kp, TX + b.toff, n, n, K, false);
        add_gemm(g1, g1t, Dy, Ey, pad(n, 16), Gv, Fv, pad(K, 16), Kp, TY + b.toff, n, n, K, false);
        add_gemm(g2, g2t, Gv, Fv, pad(K, 16), Gtx, Ftx, pad(K, 16), Kp, BX + b.boff, K, K, K, mw_pair_upper);
        add_gemm(g2, g2t, Gv, Fv, pad(K, 16), Gty, Fty, pad(K, 16), Kp, BY + b.boff, K, K, K, mw_pair_upper);
      }
      if (g1.empty()) return;
      d_ozs1 = descs.own(s1); d_ozs2 = descs.own(s2); d_ozg1 = descs.own(g1); d_ozg2 = descs.own(g2);
      d_ozs1t = descs.own(s1t); d_ozs2t = descs.own(s2t); d_ozg1t = descs.own(g1t); d_ozg2t = descs.own(g2t);
      n_ozs1 = (int)s1t.size(); n_ozs2 = (int)s2t.size(); n_ozg1 = (int)g1t.size(); n_ozg2 = (int)g2t.size();
      use_oz = true;
    }
  }
  void launch_ozaki() {
    oz_split<<<(unsigned)n_ozs1, 256, 0, stream>>>(d_ozs1, d_ozs1t);
    oz_gemm<<<(unsigned)cdiv(n_ozg1, 4), 256, 0, stream>>>(d_ozg1, d_ozg1t, n_ozg1);
    oz_split<<<(unsigned)n_ozs2, 256, 0, stream>>>(d_ozs2, d_ozs2t);
    oz_gemm<<<(unsigned)cdiv(n_ozg2, 4), 256, 0, stream>>>(d_ozg2, d_ozg2t, n_ozg2);
    HIPCHK(hipGetLastError());
  }

  bool schur_grp2 = !env_off("CLRSDP_SCHUR_GRP2");  // (per handle: tests switch it)
  bool any_grp2 = false;
  void build_fast_schur() {
    if constexpr (std::is_same<T, double>::value) {
      p_txy.tag = 1;
      p_txy.stamp = stamps;  // the SCHUR stage's start (clock stamps in the stat block)
      p_txy.tb = true;  // TXt = Vt * X^-1^T (X^-1 and Y are symmetric)
      p_ty.tag = 3;
      p_ty.stamp = stamps + 2;
      p_ty.tb = true;
      for (const LBlk& b : lb)
        if (b.K > 0) {
          p_txy.add(Vt + b.voff, b.K, Xinv + b.off, b.n, nullptr, 0, TX + b.toff, b.K, b.K, b.del, b.del);
          p_ty.add(Vt + b.voff, b.K, Y + b.off, b.n, nullptr, 0, TY + b.toff, b.K, b.K, b.del, b.del);
        }
      std::vector<PairTileDesc> ptd;
      std::vector<int> pnt;
      std::vector<SchurClusterDesc> gcd;
      int bi = 0;
      for (int c = 0; c < nc(); ++c) {
        const int j = oc[c];
        bool direct = Lc[j] == 1, grp2 = Lc[j] == 1;
        for (int l = 0; l < Lc[j] && (direct || grp2); ++l) {
          const LBlk& b = lb[bi + l];
          for (int k = 0; k < b.N; ++k) {
            direct = direct && ranks_all[rkoff_g[b.gjl] + k] == 1;
            grp2 = grp2 && ranks_all[rkoff_g[b.gjl] + k] == 2;
          }
        }
        // every sample of rank 2 (C2): the pairs kernel sums the 2 x 2 groups into S itself
        // (CLRSDP_SCHUR_GRP2=0: G and schur_gsum, for A/B)
        grp2 = grp2 && schur_grp2;
        for (int l = 0; l < Lc[j]; ++l) {
          const LBlk& b = lb[bi + l];
          if (b.K == 0) continue;
          PairTileDesc t;
          t.Vt = Vt + b.voff; t.TXt = TX + b.toff; t.TYt = TY + b.toff; t.lam = lam + b.koff;
          t.G = (direct || grp2) ? S + c_Soff[c] : BX + b.boff;
          t.ldG = grp2 ? (int)Ds[j] : b.K;
          t.grp = grp2 ? 2 : 1;
          t.pad = 0;
          t.AY = AY + b.ayoff;
          t.K = b.K; t.del = b.del; t.tile0 = 0;
          const int nt = cdiv(b.K, 64);
          pnt.push_back(nt * (nt + 1) / 2);
          ptd.push_back(t);
        }
        if (grp2) any_grp2 = true;
        if (!direct && !grp2) {
          SchurClusterDesc g;
          g.m = 1; g.N = (int)Ns[j]; g.D = (int)Ds[j]; g.blk0 = bi; g.nblk = (int)Lc[j];
          g.pair0 = 0; g.S_off = c_Soff[c];
          gcd.push_back(g);
          max_gD = std::max(max_gD, g.D);
        }
        bi += (int)Lc[j];
      }
      const std::vector<TileRef> pt2d = tile_major(pnt);
      n_ptiles = (int)pt2d.size();
      if (n_ptiles) { d_ptd = descs.own(ptd); d_pt2d = descs.own(pt2d); }
      // the fused kernel: same blocks, one workgroup per 64-row block of each
      // Taken when it fills at least half the CUs with 64 < delta <= 128 (C3 and its 2-rank
      // shards), and in its ONE form below half the CUs (small cluster counts; at delta <= 64, C2,
      // the D64 instance).  Otherwise the unfused pair, with more and smaller workgroups.
      // CLRSDP_SCHUR_FUSED=0 / 1 forces either.
      const char* ef = std::getenv("CLRSDP_SCHUR_FUSED");
      schur_fused = !(ef && ef[0] == '0') && !ptd.empty();
      int fwg = 0;
      for (const PairTileDesc& t : ptd) {
        schur_fused = schur_fused && t.del <= 128;
        fwg += cdiv(t.K, 64);
      }
      // round 6: below half the CUs, with 64 < delta, the one-tile-per-workgroup form (ONE) is
      // taken (8-cluster shard of C3: 1572-1601 -> 1607-1681 it/s against the unfused pair, three
      // A/B pairs; at C2's delta = 64 it lost 2 %: 24.9 against 22.6 us)
      // (CLRSDP_SCHUR_FUSED_ONE=0: never, =1: whenever the fused kernel runs)
      fused_one = fwg < 128 && !env_off("CLRSDP_SCHUR_FUSED_ONE");
      // (round 6, late: with every delta <= 64 the D64 instance of the ONE form -- half the MFMAs
      // of the padded one -- replaces the unfused pair below half the CUs, C2;
      // CLRSDP_SCHUR_FUSED_D64=0 keeps the padded instance wherever the fused kernel runs)
      fused_d64 = !env_off("CLRSDP_SCHUR_FUSED_D64");
      for (const PairTileDesc& t : ptd) fused_d64 = fused_d64 && t.del <= 64;
      for (const PairTileDesc& t : ptd) fused_one = fused_one && (t.del > 64 || fused_d64);
      if (env_on("CLRSDP_SCHUR_FUSED_ONE")) fused_one = true;
      if (!(ef && ef[0] == '1') && !fused_one) {
        for (const PairTileDesc& t : ptd) schur_fused = schur_fused && t.del > 64;
        schur_fused = schur_fused && fwg >= 128;
      }
      if (schur_fused) {
        std::vector<FusedPairDesc> fpd;
        std::vector<int> fnt;
        int q = 0;
        for (const LBlk& b : lb) {
          if (b.K == 0) continue;
          const PairTileDesc& t = ptd[q++];
          FusedPairDesc f;
          f.Vt = t.Vt; f.Xinv = Xinv + b.off; f.TYt = t.TYt; f.Y = Y + b.off; f.lam = t.lam;
          f.G = t.G; f.AY = t.AY;
          f.K = t.K; f.del = t.del; f.ldG = t.ldG; f.ldx = b.n; f.ldy = b.n;
          f.grp = t.grp; f.pad = 0;
          fpd.push_back(f);
          fnt.push_back(cdiv(b.K, 64));
        }
        const char* efy = std::getenv("CLRSDP_SCHUR_FUSED_Y");
        fused_y = !(efy && efy[0] == '0');
        fused_one = fused_one && fused_y;  // (instantiated with V^T Y on chip only)
        fused_d64 = fused_d64 && fused_one;   // (instantiated in the ONE form only)
        std::vector<TileRef> ft2d = tile_major(fnt);
        if (fused_one) {  // every (row block a, tile s of its share): t = a + 64 s
          std::vector<int> fnt1;
          for (int nr : fnt) fnt1.push_back(64 * (nr / 2 + 1));
          ft2d.clear();
          for (const TileRef& r : tile_major(fnt1)) {
            const int nr = fnt[r.p], a = r.t % 64, sidx = r.t / 64;
            const int nbt = (nr % 2 == 0 && a >= nr / 2) ? nr / 2 : nr / 2 + 1;
            if (a < nr && sidx < nbt) ft2d.push_back(r);
          }
        }
        n_fwg = (int)ft2d.size();
        d_fpd = descs.own(fpd);
        d_fpt2d = descs.own(ft2d);
        fused_grp2 = any_grp2;
        for (const void* k : {(const void*)schur_fused_f64<0>, (const void*)schur_fused_f64<0, true>,
                              (const void*)schur_fused_f64<0, false, true>,
                              (const void*)schur_fused_f64<0, true, true>,
                              (const void*)schur_fused_f64<0, true, false, true>,
                              (const void*)schur_fused_f64<0, true, true, true>,
                              (const void*)schur_fused_f64<0, true, false, true, true>,
                              (const void*)schur_fused_f64<0, true, true, true, true>})
          HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)schur_fused::LDS));
      }
      n_gsum = (int)gcd.size();
      if (n_gsum) d_gcd = descs.own(gcd);
    }
  }

  TrsmPlan<T> t_dx;
  void t_dxadd_init() {
    for (int c = 0; c < nc(); ++c) {
      const int D = (int)Ds[oc[c]];
      t_dx.add(S + c_Soff[c], D, dx + c_xoff[c], D, D, 1);
    }
  }

  // The LU fallback's buffers and launch plans (first switch, or set_factorization).
  //   FACTOR:  S_j[perm_j] = L_j U_j (getrf); W1_j = L_j^-1 B_j[perm_j]; W2_j = U_j^-T B_j;
  //            slab_j = W2_j^T W1_j; Q = sum_j slab_j; Q[perm] = L_Q U_Q     (MPMP.jl:1429-1505)
  //   solves:  t_j = L_j^-1 rhs_j[perm_j]; u = sum_j W2_j^T t_j; dy = U_Q^-1 L_Q^-1 (p - u)[perm];
  //            dx_j = U_j^-1 (t_j + W1_j dy)                                  (MPMP.jl:1743-1776)
  //   X^-1:    X_b[perm_b] = L_b U_b; X_b^-1 = U_b^-1 L_b^-1 (P_b I)          (approx_inv!, 781)
  // the on-chip panel of getrf_batched bounds the LU fallback (fp64 ~624, dd ~312, qd ~156)
  bool lu_fits() const {
    int nmax = (int)n_y;
    for (int c = 0; c < nc(); ++c) nmax = std::max(nmax, (int)Ds[oc[c]]);
    for (const LBlk& b : lb) nmax = std::max(nmax, b.n);
    return getrf_lds_bytes<T, LuPlan<T>::NB>(nmax) <= LDS_MAX - 4096;
  }
  void build_lu_plans() {
    if (lu_built) return;
    if (!lu_fits())
      throw ClrsdpError{CLRSDP_E_ARG, "LU factorization: a matrix is too large for the on-chip panel of getrf_batched"};
    try {
      build_lu_plans_();
    } catch (...) {  // transactional: no half-built plans or buffers survive a failure
      for (LuPlan<T>* l : {&lu_S, &lu_Q, &lu_X}) l->h.clear();
      for (PermPlan<T>* q : {&pm_B, &pm_rhs, &pm_r, &pm_I}) q->h.clear();
      for (TrsmPlan<T>* t : {&tl_W1, &tl_W2, &tl_t, &tl_dx, &tl_Q1, &tl_Q2, &tl_X1, &tl_X2}) t->h.clear();
      for (GemmPlan<T>* g : {&lq_slab, &lq_Wt}) g->clear();
      if (lperm) (void)hipFree(lperm);
      if (W2m) (void)hipFree(W2m);
      lperm = nullptr;
      W2m = nullptr;
      throw;
    }
  }
  void build_lu_plans_() {
    int64_t np = nx + n_y;
    for (const LBlk& b : lb) np += b.n;
    lperm = dmalloc<int>(std::max<int64_t>(np, 1));
    W2m = dmalloc<T>(std::max<int64_t>(nB, 1));
    const int ny = (int)n_y;
    for (int c = 0; c < nc(); ++c) {
      const int D = (int)Ds[oc[c]];
      T* Sc = S + c_Soff[c];
      T* Wc = Wm + c_Boff[c];
      T* W2c = W2m + c_Boff[c];
      const T* Bc = Bm + c_Boff[c];
      int* pc = lperm + c_xoff[c];
      const int64_t xo = c_xoff[c];
      lu_S.add(Sc, pc, D, D);
      pm_B.add(Bc, D, Wc, D, pc, D, ny);                                          // B_j[perm_j]
      tl_W1.add(Sc, D, Wc, D, D, ny);                                             // L_j^-1 (.)
      tl_W2.add(Sc, D, W2c, D, D, ny);                                            // U_j^-T B_j
      lq_slab.add(W2c, D, Wc, D, nullptr, 0, Qslab + (int64_t)c * n_y * n_y, ny, ny, ny, D);
      pm_rhs.add(rhs + xo, D, tvec + xo, D, pc, D, 1);                            // rhs_j[perm_j]
      tl_t.add(Sc, D, tvec + xo, D, D, 1);
      lq_Wt.add(W2c, D, tvec + xo, D, nullptr, 0, pslab + (int64_t)c * n_y, ny, ny, 1, D);
      tl_dx.add(Sc, D, dx + xo, D, D, 1);                                         // U_j^-1 (.)
    }
    int* qp = lperm + nx;
    lu_Q.add(Qf, qp, ny, ny);
    pm_r.add(uvec, ny, dyv, ny, qp, ny, 1);
    tl_Q1.add(Qf, ny, dyv, ny, ny, 1);
    tl_Q2.add(Qf, ny, dyv, ny, ny, 1);
    int* xp = qp + n_y;
    for (const LBlk& b : lb) {
      lu_X.add(tA + b.off, xp, b.n, b.n);
      pm_I.add(nullptr, 0, Xinv + b.off, b.n, xp, b.n, b.n);
      tl_X1.add(tA + b.off, b.n, Xinv + b.off, b.n, b.n, b.n);
      tl_X2.add(tA + b.off, b.n, Xinv + b.off, b.n, b.n, b.n);
      xp += b.n;
    }
    lq_slab.ta = lq_Wt.ta = true;
    for (TrsmPlan<T>* t : {&tl_W1, &tl_t, &tl_Q1, &tl_X1}) t->mode = 1;
    for (TrsmPlan<T>* t : {&tl_W2, &tl_dx, &tl_Q2, &tl_X2}) t->mode = 2;
    for (LuPlan<T>* l : {&lu_S, &lu_Q, &lu_X}) l->finalize();
    for (PermPlan<T>* q : {&pm_B, &pm_rhs, &pm_r, &pm_I}) q->finalize();
    for (TrsmPlan<T>* t : {&tl_W1, &tl_W2, &tl_t, &tl_dx, &tl_Q1, &tl_Q2, &tl_X1, &tl_X2}) t->finalize();
    lq_slab.finalize();
    lq_Wt.finalize();
    lu_built = true;
  }
  void set_factorization(int flags) override {
    if (inflight) throw ClrsdpError{CLRSDP_E_STATE, "set_factorization with loop bodies in flight"};
    if (flags & ~(CLRSDP_FACT_FALLBACK | CLRSDP_FACT_LU_SQ | CLRSDP_FACT_LU_X))
      throw ClrsdpError{CLRSDP_E_ARG, "unknown factorization flags"};
    if (flags & (CLRSDP_FACT_LU_SQ | CLRSDP_FACT_LU_X)) build_lu_plans();
    if (flags != fact_flags) drop_graphs();
    fact_flags = flags;
  }
  int get_factorization() const override { return fact_flags; }

  // ---------------- host <-> device conversion
  void put(T* dst, const double* planes, int64_t nplane, int64_t first, int64_t count) {
    if (count <= 0) return;
    std::vector<T> tmp(count);
    for (int64_t i = 0; i < count; ++i) Num<T>::pack(planes, nplane, first + i, &tmp[i]);
    HIPCHK(hipMemcpyAsync(dst, tmp.data(), count * sizeof(T), hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  void get(const T* src, double* planes, int64_t nplane, int64_t first, int64_t count) {
    if (count <= 0) return;
    std::vector<T> tmp(count);
    HIPCHK(hipMemcpyAsync(tmp.data(), src, count * sizeof(T), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    for (int64_t i = 0; i < count; ++i) Num<T>::unpack(tmp[i], planes, nplane, first + i);
  }

  void upload(const double* Vh, const double* lamh, const double* Bh, const double* ch,
              const double* bh, const double* Ch) override {
    for (const LBlk& b : lb) {
      put(V + b.voff, Vh, tot_V, voff_g[b.gjl], (int64_t)b.del * b.K);
      put(lam + b.koff, lamh, tot_K, koff_g[b.gjl], b.K);
      if (fast_schur && b.K > 0) {  // V^T for the fused Schur path (fp64: one plane)
        std::vector<double> vt((size_t)b.del * b.K);
        const double* src = Vh + voff_g[b.gjl];
        for (int i = 0; i < b.del; ++i)
          for (int p = 0; p < b.K; ++p) vt[p + (size_t)i * b.K] = src[i + (size_t)p * b.del];
        put(Vt + b.voff, vt.data(), (int64_t)vt.size(), 0, (int64_t)vt.size());
      }
    }
    for (int c = 0; c < nc(); ++c) {
      const int j = oc[c];
      put(Bm + c_Boff[c], Bh, tot_B, Boff_g[j], Ds[j] * n_y);
      put(cvec + c_xoff[c], ch, tot_x, xoff_g[j], Ds[j]);
    }
    put(bvec, bh, n_y, 0, n_y);
    hasC = (Ch != nullptr);
    if (hasC)
      for (const LBlk& b : lb) put(Cm + b.off, Ch, tot_blk, blkoff_g[b.gjl], (int64_t)b.n * b.n);
    uploaded = true;
  }

  void set_state(const double* xh, const double* Xh, const double* yh, const double* Yh) override {
    dy_dot_ready = false;  // (a new state: CORRECTOR_R sums <X + dX, Y + dY> itself)
    for (int c = 0; c < nc(); ++c) put(x + c_xoff[c], xh, tot_x, xoff_g[oc[c]], Ds[oc[c]]);
    for (const LBlk& b : lb) {
      put(X + b.off, Xh, tot_blk, blkoff_g[b.gjl], (int64_t)b.n * b.n);
      put(Y + b.off, Yh, tot_blk, blkoff_g[b.gjl], (int64_t)b.n * b.n);
    }
    put(y, yh, n_y, 0, n_y);
    refresh_xy_part();
    HIPCHK(hipStreamSynchronize(stream));
  }
  void get_state(double* xh, double* Xh, double* yh, double* Yh) override {
    if (xh)
      for (int c = 0; c < nc(); ++c) get(x + c_xoff[c], xh, tot_x, xoff_g[oc[c]], Ds[oc[c]]);
    for (const LBlk& b : lb) {
      if (Xh) get(X + b.off, Xh, tot_blk, blkoff_g[b.gjl], (int64_t)b.n * b.n);
      if (Yh) get(Y + b.off, Yh, tot_blk, blkoff_g[b.gjl], (int64_t)b.n * b.n);
    }
    if (yh) get(y, yh, n_y, 0, n_y);
  }

  // ---------------- exchange
  // Partials are written to xsend[0..cnt); after the exchange rank r's copy is at
  // xrecv[r*cnt..].  world == 1: xrecv == xsend, nothing to do.
  void exchange(int tag, int64_t cnt) {
    if (comm) {  // native: one all-gather on the library stream (graph-capturable)
      RCCLCHK(rccl().all_gather(xsend, xrecv, (size_t)(cnt * (int64_t)sizeof(T)), ncclUint8, comm,
                                stream));
      return;
    }
    if (world == 1) return;
    if (!xfn) throw ClrsdpError{CLRSDP_E_EXCHANGE, "world_size > 1 but no exchange registered"};
    const int rc = xfn(xctx, tag, cnt * (int64_t)sizeof(T), (void*)stream);
    if (rc != 0) throw ClrsdpError{CLRSDP_E_EXCHANGE, "exchange callback failed"};
  }
  // reduce slot `slot` of every rank's partial vector (length cnt) in rank order into dst
  // rank-ordered reduction of slot `slot` of every rank's partials into sc[dst]; folded into
  // the next scalar_kernel launch (flush_scalars() at the latest, before xsend is reused)
  std::vector<FoldRed<T>> pend;
  void reduce_ranks(int64_t cnt, int64_t slot, int op, int dst) {
    pend.push_back(FoldRed<T>{xrecv + slot, cnt, world, op, dst, 0});
  }
  void fold(const T* src, int cnt, int op, int dst) {
    pend.push_back(FoldRed<T>{src, 1, cnt, op, dst, 0});
  }
  void flush_scalars() {
    if (!pend.empty()) scalars(nullptr, 0, -1);
  }

  // ---------------- kernels shorthands
  // out = a*A + b*B over all local blocks (flat), then += s I if scal
  void blk_lin(T* out, const T* A, double a, const T* B_, double b, const T* scal = nullptr,
               double sm = 1.0) {
    if (!nb()) return;
    if (!(scal && A == out && a == 1.0 && !B_))
      vec_lin<T><<<std::min<unsigned>(cdiv(nblk_el, 256), 4096), 256, 0, stream>>>(out, A, a, B_, b, nullptr, 0.0, nblk_el);
    if (scal) diag_add<T><<<nb(), 128, 0, stream>>>(d_blk, out, scal, sm);
  }
  void vlin(T* out, const T* a_, double ca, const T* b_, double cb, const T* c_, double cc,
            int64_t n) {
    if (n > 0) vec_lin<T><<<cdiv(n, 256), 256, 0, stream>>>(out, a_, ca, b_, cb, c_, cc, n);
  }
  void copy_guarded(T* dst, const T* src, int64_t n) {
    if (n > 0)
      vec_copy_guard<T><<<std::min<unsigned>(cdiv(n, 256), 2048), 256, 0, stream>>>(dst, src, n, info + info_H);
  }
  // two guarded copies in one launch (16-byte moves)
  void copy_guarded2(T* d0, const T* s0, int64_t n0, T* d1, const T* s1, int64_t n1) {
    if (n0 <= 0 && n1 <= 0) return;
    auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if (n0 <= 0 || !a16(d0) || !a16(s0) || (n1 > 0 && (!a16(d1) || !a16(s1)))) {
      copy_guarded(d0, s0, n0);
      copy_guarded(d1, s1, n1);
      return;
    }
    const long long b0 = (long long)n0 * (long long)sizeof(T), b1 = n1 > 0 ? (long long)n1 * (long long)sizeof(T) : 0;
    const long long chunks = std::max(b0, b1) / 16 + 1;
    const unsigned g = (unsigned)std::min<long long>((chunks + 255) / 256, 1024);
    copy_guard2<<<g, 256, 0, stream>>>(d0, s0, b0, n1 > 0 ? d1 : nullptr, s1, b1, info + info_H);
  }
  void fill(T* out, double v, int64_t n) {
    if (n > 0) vec_fill<T><<<cdiv(n, 256), 256, 0, stream>>>(out, v, n);
  }
  int sym_pairs = 0;  // lower 32x32 tiles of the largest local block (blk_sym_tiles grid)
  void sym(T* out, const T* Zm, int mode, bool only_m = false) {
    if (only_m) {
      if (n_blk_m) blk_sym2<T><<<dim3(n_blk_m, 32), 128, 0, stream>>>(d_blk_m, out, Zm, mode);
    } else if (std::is_same<T, double>::value && mode == 0 && nb() && sym_pairs) {
      // (fp64: coalesced tile pairs; CLRSDP_SYM_TILES=0 keeps blk_sym2)
      blk_sym_tiles<<<dim3(nb(), sym_pairs), 256, 0, stream>>>(
          d_blk, reinterpret_cast<double*>(out), reinterpret_cast<const double*>(Zm));
    } else if (nb()) {
      blk_sym2<T><<<dim3(nb(), 32), 128, 0, stream>>>(d_blk, out, Zm, mode);
    }
  }
  static T limbs(const double* l) {
    T v = T(l[0]);
    for (int i = 1; i < Num<T>::W && i < 4; ++i) v += T(l[i]);
    return v;
  }
  ScalarParams<T> sparams(const clrsdp_params* prm, int pd_feas) {
    ScalarParams<T> p{};
    p.beta_inf = limbs(prm->beta_infeasible);
    p.beta_feas = limbs(prm->beta_feasible);
    p.gamma = limbs(prm->gamma);
    p.b0 = limbs(prm->b0);
    p.gap_thr = gap_thr;
    p.p_thr = p_thr;
    p.d_thr = d_thr;
    p.need_p = need_p;
    p.need_d = need_d;
    p.dim = dimtot;
    p.pd_feas = pd_feas;
    static const int fold_all = env_off("CLRSDP_FOLD_ALL") ? 0 : 1;
    p.fold_all = fold_all;
    return p;
  }
  void set_control(const clrsdp_control* c) override {
    if (inflight) throw ClrsdpError{CLRSDP_E_STATE, "set_control with loop bodies in flight"};
    gap_thr = limbs(c->duality_gap_threshold);
    p_thr = limbs(c->primal_error_threshold);
    d_thr = limbs(c->dual_error_threshold);
    need_p = c->need_primal_feasible != 0;
    need_d = c->need_dual_feasible != 0;
    // the thresholds travel by value in the ScalarParams of the captured scalar launches, so
    // every graph captured with the previous ones is stale
    drop_graphs();
  }
  bool zero_cy = false, zero_info = false;
  // ---- scalar slots + status words: one device block, one pinned host mirror
  char* stat_dev = nullptr;
  char* stat_host = nullptr;
  size_t stat_bytes = 0, stat_info_off = 0, stat_stamp_off = 0;
  unsigned long long* stamps = nullptr;
  void stat_alloc() {
    stat_info_off = ((SC_COUNT * sizeof(T)) + 63) / 64 * 64;
    // + the OR (update guard), then the SCHUR clock stamps (8-byte aligned)
    stat_stamp_off = (stat_info_off + (info_count + 1) * sizeof(int) + 7) / 8 * 8;
    stat_bytes = stat_stamp_off + 6 * sizeof(unsigned long long);
    stat_dev = dmalloc<char>(stat_bytes);
    HIPCHK(hipHostMalloc((void**)&stat_host, stat_bytes, hipHostMallocDefault));
    sc = reinterpret_cast<T*>(stat_dev);
    info = reinterpret_cast<int*>(stat_dev + stat_info_off);
    stamps = reinterpret_cast<unsigned long long*>(stat_dev + stat_stamp_off);
  }
  // copy scalars + status to the host mirror and wait
  void stat_fetch() {
    HIPCHK(hipMemcpyAsync(stat_host, stat_dev, stat_bytes, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  void scalars(const clrsdp_params* prm, int pd_feas, int which) {
    ScalarParams<T> p = prm ? sparams(prm, pd_feas) : ScalarParams<T>{};
    p.zero_cy = zero_cy ? 1 : 0;
    p.zero_n = zero_info ? info_count - 1 : 0;  // status words of this iteration (not the halt word)
    p.zero_ptr = info;
    p.halt_ptr = zero_info ? info + info_H : nullptr;  // which == 0 at the start of a loop body
    p.stamps = zero_info ? stamps : nullptr;
    p.guard = info;
    p.nguard = info_count;
    zero_info = false;
    size_t q = 0;
    while (q < pend.size() || q == 0) {  // at most 6 folded reductions per launch
      const size_t cnt = std::min<size_t>(6, pend.size() - q);
      p.nred = (int)cnt;
      for (size_t i = 0; i < cnt; ++i) p.red[i] = pend[q + i];
      q += cnt;
      const bool last = q >= pend.size();
      scalar_kernel<T><<<1, 64, 0, stream>>>(sc, p, last ? which : -1);
      p.zero_n = 0;
      if (last) break;
    }
    pend.clear();
  }
  // local block-sum (op 0/1) or block-max (op 2) into *dst
  static constexpr int RED_G = 256;  // fixed chunking of the flat reductions (deterministic)
  void local_blk_reduce(const T* A, const T* B_, const T* dA, const T* dB, int op, T* dst) {
    if (nb()) {
      flat_reduce<T><<<RED_G, 256, 0, stream>>>(A, B_, dA, dB, nblk_el, op, bpart);
      vec_reduce_tree(bpart, RED_G, op, dst);
    } else {
      fill(dst, 0.0, 1);
    }
  }

  // one-workgroup fixed-tree reduction of n <= 256 partials
  void vec_reduce_tree(const T* in, int n, int op, T* dst) {
    vec_reduce<T><<<1, vec_reduce_threads<T>(), 0, stream>>>(in, in, n, op == 2 ? 2 : 3, dst);
  }

  // trace_A with the products U already in TX -> val (tval) -> aggregate
  void trace_aggregate(const T* val, const T* in, double c_in, const T* in2, double c_in2,
                       double c_agg, T* out) {
    if (nx > 0)
      tuple_aggregate<T><<<cdiv(nx, 256), 256, 0, stream>>>(d_td, nc(), d_tb, rsums, lam, val, in,
                                                            c_in, in2, c_in2, c_agg, out, nx);
  }
  void colsums() {
    if (n_pair) {
      dim3 g(cdiv(max_K, 4), n_pair);
      colsum_dot<T><<<g, 256, 0, stream>>>(d_pair, TU, V, tval);
    }
  }
  void weighted_A(const T* a, const GemmPlan<T>& plan, T* out, double beta = 0.0) {
    if (wa_fused) {
      (a == x ? p_wA_Ps : p_wA_dXs).launch(stream, 1.0, beta);
      return;
    }
    if (n_pair) {
      dim3 g(64, n_pair);
      scale_cols<T><<<g, 256, 0, stream>>>(d_scale, V, lam, ksamp, a, TW);
    }
    plan.launch(stream, 1.0, beta);
    if (anyMgt1) sym(out, out, 1, true);  // Symmetric(.) on blocks with m != 1 (MPMP.jl:1671-1674)
  }

  // ---------------- stages
  void st_mu_r(const clrsdp_params* prm, int pd_feas) {
    mu_scalars(prm, pd_feas);
    if (!fuse_r) mu_r_gemm();
  }
  // (round 6) a loop body at fp64 forms R = mu_p I - XY in XINV's launch, beside
  // X^-1 = L^-T L^-1: a mixed batch (gemm_f64_dyn, the mu_p diagonal from the scalar slot) instead
  // of a 128^3 GEMM launch of its own on the critical path before chol_inv(X, Y) -- R is first
  // read by the predictor's Z after SCHUR.  CLRSDP_FUSE_R=0 keeps the separate launch.
  bool fuse_r = false;
  GemmPlan<T> p_xir;
  // mu = <X,Y>/dim, mu_p (and the status words cleared, the halt word decided)
  void mu_scalars(const clrsdp_params* prm, int pd_feas) {
    blk_dot(X, Y, nullptr, nullptr, 0, SC_DOT_XY, 1, upart);
    zero_info = true;  // the first scalar launch of an iteration clears the status words
    scalars(prm, pd_feas, 0);
  }
  void mu_r_gemm() { gemm_diag(p_XY, -1.0, 0.0, SC_MU_P); }  // R = mu_p I - XY
  // sum/max over the local blocks into sc[slot], all-gathered and rank-reduced when world > 1;
  // part: the flat_reduce partials are already there (<X,Y>, from update_state)
  void blk_dot(const T* A, const T* B_, const T* dA, const T* dB, int op, int slot, int tag,
               const T* part = nullptr) {
    if (world == 1 && nb()) {
      if (!part) flat_reduce<T><<<RED_G, 256, 0, stream>>>(A, B_, dA, dB, nblk_el, op, bpart);
      fold(part ? part : bpart, RED_G, op == 2 ? 2 : 0, slot);  // folded into the next scalar launch
      return;
    }
    if (part && nb()) vec_reduce_tree(part, RED_G, op, xsend);
    else local_blk_reduce(A, B_, dA, dB, op, xsend);
    exchange(tag, 1);
    reduce_ranks(1, 0, op == 2 ? 2 : 0, slot);
  }
  // plan.launch + "s I" on the block diagonals (fused into the fp64 GEMM epilogue)
  void gemm_diag(const GemmPlan<T>& plan, double alpha, double beta, int slot) {
    if constexpr (std::is_same<T, double>::value) {
      plan.launch(stream, alpha, beta, sc + slot, 1.0);
    } else {
      plan.launch(stream, alpha, beta);
      if (nb()) diag_add<T><<<nb(), 128, 0, stream>>>(d_blk, R, sc + slot, 1.0);
    }
  }
  void st_xinv() {
    if (reg_blk) {  // L_X^-1 and L_Y^-1 on chip in one launch, X^-1 = L^-T L^-1 on MFMA
      ci_XY.launch(stream, info);
      if (lu_x()) {
        xinv_lu();
        if (fuse_r) mu_r_gemm();
      } else if (fuse_r) {
        p_xir.launch(stream, 1.0, 0.0);  // {X^-1 = L^-T L^-1 | R = mu_p I - XY}
      } else {
        q_xinv.launch(stream, 1.0, 0.0);
      }
      return;
    }
    if (fuse_r) mu_r_gemm();
    blk_lin(LX, X, 1.0, nullptr, 0.0);
    f_X.potrf(stream, info);
    if (lu_x()) {
      xinv_lu();
      return;
    }
    if (nb()) blk_identity<T><<<nb(), 256, 0, stream>>>(d_blk, tA);
    t_Linv.launch(stream, false);             // tA = L^-1
    p_xinv.launch(stream, 1.0, 0.0);          // X^-1 = L^-T L^-1
  }
  // approx_inv! (MPMP.jl:781, 788): X_b^-1 = U_b^-1 L_b^-1 P_b by pivoted LU (the Cholesky factor
  // above stays: the step length needs it, cho! MPMP.jl:1846)
  void xinv_lu() {
    blk_lin(tA, X, 1.0, nullptr, 0.0);
    lu_X.launch(stream, info + info_L0);
    pm_I.launch(stream, true);                // Xinv = P I
    tl_X1.launch(stream, false);              // L^-1 (P I)
    tl_X2.launch(stream, true);               // U^-1 (L^-1 P I)
  }
  void st_schur() {
    if constexpr (std::is_same<T, double>::value) {
      if (fast_schur) {
        if (!schur_fused) p_txy.launch(stream, 1.0, 0.0);
        if (ty_ahead) {  // V^T Y came from the side stream
          HIPCHK(hipStreamWaitEvent(stream, ev_ty, 0));
          ty_ahead = false;
        } else if (!(schur_fused && fused_y)) {
          p_ty.launch(stream, 1.0, 0.0);
        }
        // the fused kernel writes the lower triangle of S only when every reader takes that
        // triangle (the fp64 Cholesky FACTOR: chol_inv_tiles, and L21^T = L11^-1 S21^T); the
        // pivoted LU and the rank-group sums read all of it.  CLRSDP_SCHUR_FULL=1 for A/B
        static const bool force_full = env_on("CLRSDP_SCHUR_FULL");
        const bool full = force_full || !fac2 || n_gsum > 0 || lu_sq();
        s_lower = schur_fused && !full;
        if (schur_fused && fused_d64 && fused_grp2)
          schur_fused_f64<0, true, true, true, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused && fused_d64)
          schur_fused_f64<0, true, false, true, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused && fused_one && fused_grp2)
          schur_fused_f64<0, true, true, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused && fused_one)
          schur_fused_f64<0, true, false, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused && fused_y && fused_grp2)
          schur_fused_f64<0, true, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused && fused_y)
          schur_fused_f64<0, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused && fused_grp2)
          schur_fused_f64<0, false, true><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (schur_fused)
          schur_fused_f64<0><<<n_fwg, 512, schur_fused::LDS, stream>>>(d_fpd, d_fpt2d, stamps + 4, full);
        else if (n_ptiles)
          schur_pairs_f64<16><<<n_ptiles, 256, 0, stream>>>(d_ptd, d_pt2d, stamps + 4);
        if (n_gsum) {
          dim3 g((unsigned)std::min<int64_t>(cdiv((int64_t)max_gD * max_gD, 256), 64), n_gsum);
          schur_gsum<T><<<g, 256, 0, stream>>>(d_gcd, d_sbd, rsums, BX, S);
        }
        HIPCHK(hipGetLastError());
        return;
      }
    }
    if (use_oz) {
      launch_ozaki();
    } else {
      p_s1x.launch(stream, 1.0, 0.0);
      p_s1y.launch(stream, 1.0, 0.0);
      p_s2x.launch(stream, 1.0, 0.0);
      p_s2y.launch(stream, 1.0, 0.0);
    }
    if (nb()) extract_AY<T><<<nb(), 256, 0, stream>>>(d_ayd, BY, AY);
    if (n_pairs)
      schur_assemble<T><<<cdiv(n_pairs, 256), 256, 0, stream>>>(d_scd, nc(), d_sbd, rsums, lam, BX,
                                                                 BY, S, n_pairs, mw_pair_upper ? 1 : 0);
  }
  void st_factor() {
    factor_local();
    factor_q();
  }
  // side_x21: X21 on the side stream (the loop body), joined before the first solve
  bool w_split = false;  // the last factor_local ran W1's products on aux2 (ev_w recorded)
  bool fuse_alpha = false;   // enqueue_iteration: STEP leaves alpha to UPDATE's launch
  bool alpha_fused = false;  // STEP left it (the next st_update forms it)
  void factor_local(bool side_x21 = false) {
    s_lower = false;  // S now turns into L^-1 (or the LU factors)
    w_split = false;
    // (inner timing buckets: a mixed batch counts where most of its work is; the reference's
    // chol_S / CinvB / Q split, MPMP.jl:1429-1495)
    if (lu_sq()) {                            // approx_lu! (MPMP.jl:1433-1494)
      seg(CLRSDP_INNER_CHOL_S, [&] { lu_S.launch(stream, info + info_S0); });
      seg(CLRSDP_INNER_CINVB, [&] {
        pm_B.launch(stream);
        tl_W1.launch(stream, false);          // W1_j = L_j^-1 B_j[perm_j]
        vlin(W2m, Bm, 1.0, nullptr, 0, nullptr, 0, nB);
        tl_W2.launch(stream, false);          // W2_j = U_j^-T B_j
      });
      seg(CLRSDP_INNER_Q, [&] {
        lq_slab.launch(stream, 1.0, 0.0);     // slab_j = W2_j^T W1_j
        sum_q_slabs();
      });
      return;
    }
    if (fac2) {                               // fp64: S_j <- L_j^-1 in place, W_j and Q's slabs
      seg(CLRSDP_INNER_CHOL_S, [&] { ci_S.launch(stream, info + info_S0); });  // S / S11 blocks
      seg(CLRSDP_INNER_CINVB, [&] { f_a.launch(stream, 1.0, 0.0); });          // {L21^T | W}
      // W1 = L11^-1 B1, then W1^T W1 and B2' = B2 - L21 W1: beside the S22 chain in a loop body
      const bool split = side_x21 && nc2 && aux2 != stream;
      w_split = split;
      auto w_work = [&] {
        seg(CLRSDP_INNER_CINVB, [&] { f_w.launch(stream, 1.0, 0.0); });
        seg(CLRSDP_INNER_Q, [&] { f_w2.launch(stream, 1.0, 0.0); });
      };
      if (split) {
        HIPCHK(hipEventRecord(ev_fa, stream));
        HIPCHK(hipStreamWaitEvent(aux2, ev_fa, 0));
        {
          StreamSwitch on_aux2(stream, aux2);
          w_work();
        }
        HIPCHK(hipEventRecord(ev_w, aux2));
      } else {
        w_work();
      }
      seg(CLRSDP_INNER_CHOL_S, [&] { f_b.launch(stream, 1.0, 0.0); });         // S22 - L21 L21^T | W^T W
      if (nc2) {
        seg(CLRSDP_INNER_CHOL_S, [&] { ci_S22.launch(stream, info + info_S0 + nc()); });
        if (side_x21) {
          // X21 on the second side stream when W1's products went there (it is idle by now), so
          // that the first side stream is free for the right-hand side and chol(Q) as soon as Q
          // is summed (CLRSDP_X21_AUX2=0: on the first side stream, behind them)
          static const bool x21_aux2 = !env_off("CLRSDP_X21_AUX2");
          const hipStream_t xs = split && x21_aux2 ? aux2 : aux;
          const hipStream_t main_s = stream;
          HIPCHK(hipEventRecord(ev_x2, main_s));
          HIPCHK(hipStreamWaitEvent(xs, ev_x2, 0));
          {
            StreamSwitch on_side(stream, xs);  // restored on scope exit, also when a launch throws
            seg(CLRSDP_INNER_CHOL_S, [&] {
              f_x1.launch(xs, 1.0, 0.0);
              f_x2.launch(xs, -1.0, 0.0);
            });
          }
          HIPCHK(hipEventRecord(ev_x21, xs));
          pending_x21 = true;
        } else {
          seg(CLRSDP_INNER_CHOL_S, [&] {
            f_x1.launch(stream, 1.0, 0.0);
            f_x2.launch(stream, -1.0, 0.0);
          });
        }
        if (split) HIPCHK(hipStreamWaitEvent(stream, ev_w, 0));
        seg(CLRSDP_INNER_CINVB, [&] { f_c.launch(stream, 1.0, 0.0); });
        seg(CLRSDP_INNER_Q, [&] { f_d.launch(stream, 1.0, 1.0); });
      }
      seg(CLRSDP_INNER_Q, [&] { sum_q_slabs(); });
      return;
    }
    if (reg_S) {                              // S_j <- L_j^-1 in place; W_j = L_j^-1 B_j (MFMA)
      seg(CLRSDP_INNER_CHOL_S, [&] { ci_S.launch(stream, info + info_S0); });
      seg(CLRSDP_INNER_CINVB, [&] { q_W.launch(stream, 1.0, 0.0); });
    } else {
      seg(CLRSDP_INNER_CHOL_S, [&] { f_S.potrf(stream, info + info_S0); });
      if (s_split) {  // L_j^-1 for the GEMV solves, beside W_j and the Q chain
        const hipStream_t ls = side_x21 && aux2 ? aux2 : stream;  // (a loop body only)
        if (ls != stream) {
          HIPCHK(hipEventRecord(ev_sp, stream));
          HIPCHK(hipStreamWaitEvent(ls, ev_sp, 0));
        }
        if (!t_Sinv.vec_rhs())
          HIPCHK(hipMemcpyAsync(SLi, SLid, (size_t)s_len * sizeof(T), hipMemcpyDeviceToDevice, ls));
        t_Sinv.launch(ls, false);
        if (ls != stream) {
          HIPCHK(hipEventRecord(ev_sinv, ls));
          pending_sinv = true;
        }
      }
      seg(CLRSDP_INNER_CINVB, [&] {
        if (!t_W.vec_rhs()) vlin(Wm, Bm, 1.0, nullptr, 0, nullptr, 0, nB);
        t_W.launch(stream, false);            // W_j = L_j^-1 B_j
      });
    }
    seg(CLRSDP_INNER_Q, [&] {
      p_Q.launch(stream, 1.0, 0.0);           // slab_j = W_j^T W_j
      sum_q_slabs();
    });
  }
  // Q = sum_j slab_j (all-gathered over the ranks)
  void sum_q_slabs() {
    const int64_t q2 = n_y * n_y;
    // (potrf factors Q in place in Qf: the slab sum writes that copy too, one launch fewer on the
    // critical path; CLRSDP_Q_DUAL=0 keeps the separate copy)
    static const bool dual_on = !env_off("CLRSDP_Q_DUAL");
    T* q_dual = dual_on && !reg_Q && Qf ? Qf : nullptr;
    qf_fresh = q_dual != nullptr;
    if (world == 1 && nc()) {
      slab_sum4<T><<<cdiv(q2, 64), 256, 0, stream>>>(Qslab, nc(), q2, q2, Q, nullptr, 0.0, 1.0, q_dual);
    } else {
      if (nc()) slab_sum4<T><<<cdiv(q2, 64), 256, 0, stream>>>(Qslab, nc(), q2, q2, xsend);
      else fill(xsend, 0.0, q2);
      exchange(2, q2);
      slab_sum4<T><<<cdiv(q2, 64), 256, 0, stream>>>(xrecv, world, q2, q2, Q, nullptr, 0.0, 1.0, q_dual);
    }
  }
  void factor_q() {
    seg(CLRSDP_INNER_CHOL_Q, [&] { factor_q_(); });
  }
  void factor_q_() {
    const int64_t q2 = n_y * n_y;
    const bool fresh = qf_fresh;  // Qf = Q written by this iteration's slab sum
    qf_fresh = false;
    if (lu_sq()) {                            // approx_lu!(perm, Q) (MPMP.jl:1499-1505)
      if (!fresh) vlin(Qf, Q, 1.0, nullptr, 0, nullptr, 0, q2);
      lu_Q.launch(stream, info + info_Q0);
      return;
    }
    if (reg_Q) {
      ci_Q.launch(stream, info + info_Q0);    // Qf = L_Q^-1
      q_qinv.launch(stream, 1.0, 0.0);        // Q^-1 = L_Q^-T L_Q^-1
    } else {
      if (!fresh) vlin(Qf, Q, 1.0, nullptr, 0, nullptr, 0, q2);
      f_Q.potrf(stream, info + info_Q0);
      if (q_split) {  // Q^-1 = L_Q^-T L_Q^-1 with L_Q^-1 = L_Q \ I
        if (!t_Qinv.vec_rhs())
          HIPCHK(hipMemcpyAsync(QLi, QLid, (size_t)q2 * sizeof(T), hipMemcpyDeviceToDevice, stream));
        t_Qinv.launch(stream, false);
        q_qinv2.launch(stream, 1.0, 0.0);
      }
    }
  }
  void st_residuals(bool use_AY) {
    residuals_local(use_AY);
    residuals_finish();
  }
  // P, d, the p-slabs and the local error maxima (no exchange: may run on the side stream)
  void residuals_local(bool use_AY) {
    residuals_P();
    residuals_rest(use_AY);
  }
  // P = sum_i x_i A_i - X - C (the state only)
  void residuals_P() {
    weighted_A(x, p_wA_P, P, -1.0);
    if (hasC) blk_lin(P, P, 1.0, Cm, -1.0);
  }
  // d, the p-slabs, the maxima of |P| and |d| (A_Y from SCHUR when use_AY)
  void residuals_rest(bool use_AY) {
    // d = c - B y - Tr(A_* Y)
    p_By.launch(stream, 1.0, 0.0);
    if (!use_AY) {
      p_trU_Y.launch(stream, 1.0, 0.0);
      colsums();
    }
    trace_aggregate(use_AY ? AY : tval, cvec, 1.0, tmpv, -1.0, -1.0, dvec);
    // p partial = sum_j B_j^T x_j (slabs) ; local maxima of |P| and |d| into tmpsc[0..1]
    p_Btx.launch(stream, 1.0, 0.0);
    local_blk_reduce(P, nullptr, nullptr, nullptr, 2, tmpsc);
    if (nx > 0) vec_reduce<T><<<1, vec_reduce_threads<T>(), 0, stream>>>(dvec, nullptr, nx, 2, tmpsc + 1);
    else fill(tmpsc + 1, 0.0, 1);
  }
  // defer (a loop body at one rank): the three error maxima are only read by the log and the
  // loop control at UPDATE, so their folds ride in CORRECTOR_R's scalar launch instead of a launch
  // of their own on the critical path before the predictor's solves (their sources, tmpsc and p,
  // are not written again before it; with world > 1 they come from the exchange buffer, which the
  // solves' all-gathers overwrite, so they are flushed here)
  void residuals_finish(bool defer = false) {
    const int64_t k = n_y + 2;
    if (world == 1 && nc()) {  // p = b - sum_j B_j^T x_j in one launch; maxima folded
      slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, pvec, bvec, 1.0, -1.0);
      fold(tmpsc, 1, 2, SC_ERR_PMAT);
      fold(tmpsc + 1, 1, 2, SC_ERR_DVEC);
      fold(pvec, (int)n_y, 4, SC_ERR_PVEC);
      if (!defer) flush_scalars();
      return;
    }
    if (nc()) slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, xsend);
    else fill(xsend, 0.0, n_y);
    vlin(xsend + n_y, tmpsc, 1.0, nullptr, 0, nullptr, 0, 2);
    exchange(3, k);
    slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(xrecv, world, k, n_y, uvec);
    vlin(pvec, bvec, 1.0, uvec, -1.0, nullptr, 0, n_y);      // p = b - sum B^T x
    reduce_ranks(k, n_y, 2, SC_ERR_PMAT);
    reduce_ranks(k, n_y + 1, 2, SC_ERR_DVEC);
    fold(pvec, (int)n_y, 4, SC_ERR_PVEC);
    flush_scalars();
  }
  void st_direction(int tag) {
    direction_Z();
    direction_rhs();
    direction_rest(tag);
  }
  // Z = sym(X^-1 (P Y - R)) and the trace_A products U = Z V (no factorisation needed: in a
  // loop body the predictor's share runs on the side stream during FACTOR)
  void direction_Z() {
    seg(CLRSDP_INNER_Z, [&] { direction_Z_(); });
  }
  void direction_Z_() {
    if (c_Z.on) {
      c_Z.launch(stream, 1.0, -1.0);
    } else {
      p_PY.launch(stream, 1.0, -1.0);
      p_Z.launch(stream, 1.0, 0.0);
    }
    // Z is only consumed by trace_A: v^T Z v = v^T sym(Z) v, so the symmetrisation
    // (MPMP.jl:1704-1716) matters only for the off-diagonal (r != s) blocks of m > 1
    if (anyMgt1) sym(Z, Z, 0);
    if (!c_trZ.on) p_trU_Z.launch(stream, 1.0, 0.0);  // (else U stays on chip, direction_rhs_)
  }
  // rhs_x = -d - Tr(A_* Z)   (MPMP.jl:1733-1739)
  void direction_rhs() {
    seg(CLRSDP_INNER_RHS_X, [&] { direction_rhs_(); });
  }
  void direction_rhs_() {
    if (c_trZ.on) {
      c_trZ.launch(stream, 1.0, 0.0);   // rhs = -d - lambda (V^T Z V)_tt, U = Z V on chip
    } else if (trivial_tuples) {
      dim3 g(cdiv(max_K, 4), n_pair);
      colsum_rhs<T><<<g, 256, 0, stream>>>(d_pair, TU, V, lam, dvec, -1.0, nullptr, 0.0, -1.0, rhs);
    } else {
      colsums();
      trace_aggregate(tval, dvec, -1.0, nullptr, 0.0, -1.0, rhs);
    }
  }
  // the block solve (MPMP.jl:1743-1776), dX and dY
  void direction_rest(int tag) {
    seg(CLRSDP_INNER_SOLVE, [&] { direction_solves(tag); });
    // dX = P + sum_i dx_i A_i
    seg(CLRSDP_INNER_DX, [&] { weighted_A(dx, p_wA_dX, dX, 1.0); });
    if (tag == 6 && xy_ov_body && xy_ov_ok && aux != stream) {
      // the X step length beside dY and the Y one (STEP joins it)
      HIPCHK(hipEventRecord(ev_dxo, stream));
      HIPCHK(hipStreamWaitEvent(aux, ev_dxo, 0));
      c_stepX.launch(aux, 1.0, 0.0);
      e_Xs.eigmin(aux, eigX);
      HIPCHK(hipEventRecord(ev_stx, aux));
      xy_ov = true;
    }
    // dY = sym(X^-1 (R - dX Y))
    seg(CLRSDP_INNER_DY, [&] {
      if (c_dY.on) {
        dy_dot_ready = dy_dot_ok && tag == 4;
        c_dY.u.dot_part = dy_dot_ready ? reinterpret_cast<double*>(dotp) : nullptr;
        c_dY.launch(stream, -1.0, 1.0);
      } else {
        p_dXY.launch(stream, -1.0, 1.0);
        p_dY.launch(stream, 1.0, 0.0);
      }
      sym(dY, dY, 0);
    });
  }
  // the three-stage solve and dx as separate batched launches (any word type / rank count)
  void direction_solves(int tag) {
    // t_j = L_j^-1 rhs_j ;  u = sum_j W_j^T t_j ;  dy = Q^-1 (p - u) ; dx_j = L_j^-T (t_j + W_j dy)
    if (pending_x21) {  // X21 (lower-left block of L^-1) comes from the side stream
      HIPCHK(hipStreamWaitEvent(stream, ev_x21, 0));
      pending_x21 = false;
    }
    if (lu_sq()) {
      direction_solves_lu(tag);
      return;
    }
    if constexpr (std::is_same<T, double>::value) {
      if (cls_on) {  // t and the partial slabs | dy = Q^-1 (p - sum) | u and dx: three launches
        const unsigned g = (unsigned)(nc() * cls_nrb);
        cl_solve_t<<<g, 256, 0, stream>>>(d_cls, cls_nrb, (int)n_y, pslab);
        const double* src = pslab;
        int cnt = nc() * cls_nrb;
        if (world > 1) {
          slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, cnt, n_y, n_y, xsend);
          exchange(tag, n_y);
          src = xrecv;
          cnt = world;
        }
        if (pending_q) {
          HIPCHK(hipStreamWaitEvent(stream, ev_q, 0));
          pending_q = false;
        }
        slab_qsolve<<<cdiv(n_y, 64), 256, ((size_t)n_y + 256) * sizeof(double), stream>>>(
            src, cnt, n_y, (int)n_y, pvec, 1.0, -1.0, Qinv, (int)n_y, dyv);
        cl_solve_dx<<<g, 256, 0, stream>>>(d_cls, cls_nrb, (int)n_y, dyv);
        HIPCHK(hipGetLastError());
        return;
      }
    }
    if (pending_sinv) {
      HIPCHK(hipStreamWaitEvent(stream, ev_sinv, 0));
      pending_sinv = false;
    }
    if (reg_S) {
      q_t.launch(stream, 1.0, 0.0);
    } else if (s_split) {
      q_t2.launch(stream, 1.0, 0.0);
    } else {
      vlin(tvec, rhs, 1.0, nullptr, 0, nullptr, 0, nx);
      t_t.launch(stream, false);
    }
    p_Wt.launch(stream, 1.0, 0.0);
    // fp64 with the explicit Q^-1: r = p - sum of the slabs and dy = Q^-1 r in one launch
    // (slab_qsolve; CLRSDP_SLAB_QSOLVE=0 keeps slab_sum + the GEMV)
    bool fused_done = false;
    if constexpr (std::is_same<T, double>::value) {
      static const bool fused_q = [] {
        const char* e = std::getenv("CLRSDP_SLAB_QSOLVE");
        return !(e && e[0] == '0');
      }();
      const size_t lds = ((size_t)n_y + 256) * sizeof(double);
      // every workgroup re-forms all of r: cdiv(n_y, 64) x cnt x n_y slab reads in all.  Fused
      // only while those stay small (C3: 2 x 64 x 128); otherwise slab_sum forms r once
      const long long cnt_x = (world == 1 && nc()) ? nc() : world;
      const bool small_sum = (long long)cdiv(n_y, 64) * cnt_x * n_y <= (1LL << 20);
      if (reg_Q && fused_q && small_sum && lds <= 64 * 1024) {
        const double* src = pslab;
        int cnt = nc();
        if (!(world == 1 && nc())) {
          if (nc()) slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, xsend);
          else fill(xsend, 0.0, n_y);
          exchange(tag, n_y);
          src = xrecv;
          cnt = world;
        }
        if (pending_q) {
          HIPCHK(hipStreamWaitEvent(stream, ev_q, 0));
          pending_q = false;
        }
        slab_qsolve<<<cdiv(n_y, 64), 256, lds, stream>>>(src, cnt, n_y, (int)n_y, pvec, 1.0, -1.0,
                                                          Qinv, (int)n_y, dyv);
        HIPCHK(hipGetLastError());
        fused_done = true;
      }
    }
    if (!fused_done) {
      // r = p - sum_j W_j^T t_j  (-> uvec with the explicit Q^-1, -> dyv for the two solves)
      T* rv = (reg_Q || q_split) ? uvec : dyv;
      if (world == 1 && nc()) {  // one launch
        slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, rv, pvec, 1.0, -1.0);
      } else {
        if (nc()) slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, xsend);
        else fill(xsend, 0.0, n_y);
        exchange(tag, n_y);
        slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(xrecv, world, n_y, n_y, rv, pvec, 1.0, -1.0);
      }
      if (pending_q) {  // L_Q^-1 and Q^-1 are being computed on the side stream (iterate)
        HIPCHK(hipStreamWaitEvent(stream, ev_q, 0));
        pending_q = false;
      }
      if (reg_Q || q_split) {
        q_qdy.launch(stream, 1.0, 0.0);         // dy = Q^-1 r
      } else {
        t_Q.launch(stream, false);
        t_Q.launch(stream, true);
      }
    }
    // dx_j = L_j^-T (t_j + W_j dy)
    if (reg_S || s_split) {
      q_Wdy.launch(stream, 1.0, 1.0);
      (s_split ? q_dx2 : q_dx).launch(stream, 1.0, 0.0);
    } else {
      p_Wdy.launch(stream, 1.0, 1.0);
      t_dx.launch(stream, true);
    }
  }
  // the same with the LU factors (approx_solve_tril!/approx_solve_lu_precomp!/approx_solve_triu!,
  // MPMP.jl:1751-1773)
  void direction_solves_lu(int tag) {
    pm_rhs.launch(stream);                    // t_j = rhs_j[perm_j]
    tl_t.launch(stream, false);               // t_j = L_j^-1 t_j
    lq_Wt.launch(stream, 1.0, 0.0);           // slab_j = W2_j^T t_j  (B_j^T U_j^-1 t_j)
    if (world == 1 && nc()) {
      slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, uvec, pvec, 1.0, -1.0);
    } else {
      if (nc()) slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(pslab, nc(), n_y, n_y, xsend);
      else fill(xsend, 0.0, n_y);
      exchange(tag, n_y);
      slab_sum4<T><<<cdiv(n_y, 64), 256, 0, stream>>>(xrecv, world, n_y, n_y, uvec, pvec, 1.0, -1.0);
    }
    if (pending_q) {
      HIPCHK(hipStreamWaitEvent(stream, ev_q, 0));
      pending_q = false;
    }
    pm_r.launch(stream);                      // dy = (p - u)[perm_Q]
    tl_Q1.launch(stream, false);              // L_Q^-1
    tl_Q2.launch(stream, true);               // U_Q^-1
    p_Wdy.launch(stream, 1.0, 1.0);           // dx_j = t_j + W1_j dy
    tl_dx.launch(stream, true);               // dx_j = U_j^-1 (.)
  }
  void st_corrector_r(const clrsdp_params* prm, int pd_feas) {
    if (dy_dot_ready) fold(dotp, dy_dot_cnt, 0, SC_DOT_XDY);  // (from the predictor's dY chain)
    else blk_dot(X, Y, dX, dY, 1, SC_DOT_XDY, 5);
    dy_dot_ready = false;
    scalars(prm, pd_feas, 1);
    if constexpr (std::is_same<T, double>::value) {
      // R still holds mu_p I - XY from MU_R (the predictor only reads it), so one GEMM:
      // R = (mu_p I - XY) - dX dY + (mu_c - mu_p) I, without forming XY again
      gemm_diag(p_dXdY, -1.0, 1.0, SC_DMU);
    } else {  // multi-word: the reference's order of operations (MPMP.jl:1209-1214)
      p_XY.launch(stream, -1.0, 0.0);
      gemm_diag(p_dXdY, -1.0, 1.0, SC_MU_C);    // R = mu_c I - XY - dX dY
    }
  }
  void st_step(const clrsdp_params* prm, int pd_feas) {
    if (reg_blk) {
      // L_X^-1, L_Y^-1 from the X^-1 stage;  M = L^-1 dM L^-T on MFMA; one eigen launch
      if (xy_ov) {  // (the X half is on the side stream since dX)
        c_stepY.launch(stream, 1.0, 0.0);
        e_Ys.eigmin(stream, eigY);
        HIPCHK(hipStreamWaitEvent(stream, ev_stx, 0));
        xy_ov = false;
      } else {
        if (c_step.on) {
          c_step.launch(stream, 1.0, 0.0);        // X and Y blocks together, one launch
        } else {
          q_sx1.launch(stream, 1.0, 0.0);         // X and Y blocks together
          q_sx2.launch(stream, 1.0, 0.0);
        }
        e_XY.eigmin(stream, eigX);
      }
    } else {
      // X: L_X from the X^-1 stage
      blk_lin(tA, dX, 1.0, nullptr, 0.0);
      t_sX1.launch(stream, false);
      sym(tB, tA, 2);
      t_sX2.launch(stream, false);
      e_X.eigmin(stream, eigX);
      // Y
      blk_lin(LY, Y, 1.0, nullptr, 0.0);
      f_Y.potrf(stream, info + info_Y0);
      blk_lin(tA, dY, 1.0, nullptr, 0.0);
      t_sY1.launch(stream, false);
      sym(tB, tA, 2);
      t_sY2.launch(stream, false);
      e_Y.eigmin(stream, eigY);
    }
    if (world == 1 && nb() && fuse_alpha) {
      // (a loop body: the minima and alpha are formed by UPDATE's update_state, one launch less)
      flush_scalars();
      alpha_fused = true;
      return;
    }
    if (world == 1 && nb()) {  // min over the blocks straight into the scalar slots
      fold(eigX, nb(), 3, SC_MINEIG_X);
      fold(eigY, nb(), 3, SC_MINEIG_Y);
    } else {
      if (nb()) {
        ordered_reduce<T><<<1, 1, 0, stream>>>(eigX, nb(), 1, 3, xsend);
        ordered_reduce<T><<<1, 1, 0, stream>>>(eigY, nb(), 1, 3, xsend + 1);
      } else {
        fill(xsend, 1e300, 2);  // no local blocks: neutral element of min
      }
      // + this rank's failure bits: every rank guards its update and reports (and falls back)
      // on the OR over all ranks, so the ranks stay in step
      status_bits<T><<<1, 256, 0, stream>>>(info, nb(), nc() + nc2, info_S0, info_Q0, info_L0, xsend + 2);
      exchange(8, 3);
      status_gather<T><<<1, 64, 0, stream>>>(xrecv, world, 3, 2, info + info_G);
      reduce_ranks(3, 0, 3, SC_MINEIG_X);
      reduce_ranks(3, 1, 3, SC_MINEIG_Y);
    }
    scalars(prm, pd_feas, 2);
  }
  void objectives(const clrsdp_params* prm, int pd_feas, int which = 3) {
    zero_cy = !hasC;
    if (world == 1) {
      if (nx > 0) vec_reduce<T><<<1, vec_reduce_threads<T>(), 0, stream>>>(cvec, x, nx, 0, sc + SC_DOT_CX);
      else fill(sc + SC_DOT_CX, 0.0, 1);
      if (hasC) local_blk_reduce(Cm, Y, nullptr, nullptr, 0, sc + SC_DOT_CY);
    } else {
      if (nx > 0) vec_reduce<T><<<1, vec_reduce_threads<T>(), 0, stream>>>(cvec, x, nx, 0, xsend);
      else fill(xsend, 0.0, 1);
      if (hasC) local_blk_reduce(Cm, Y, nullptr, nullptr, 0, xsend + 1);
      else fill(xsend + 1, 0.0, 1);
      exchange(9, 2);
      reduce_ranks(2, 0, 0, SC_DOT_CX);
      reduce_ranks(2, 1, 0, SC_DOT_CY);
    }
    vec_reduce<T><<<1, vec_reduce_threads<T>(), 0, stream>>>(bvec, y, n_y, 0, sc + SC_DOT_BY);
    scalars(prm, pd_feas, which);
    zero_cy = false;
  }
  void st_update(const clrsdp_params* prm, int pd_feas) {
    // one launch updates x, y, X, Y (guarded by the status words: no update after a failed
    // factorisation) and leaves the partial sums <X,Y> (next MU_R), <c,x> and <b,y>
    StepAlpha<T> sa{};
    if (alpha_fused) {
      sa.eigX = eigX;
      sa.eigY = eigY;
      sa.nb = nb();
      sa.pd_feas = pd_feas;
      sa.gamma = limbs(prm->gamma);
      sa.sc = sc;
      sa.sx = SC_MINEIG_X;
      sa.sy = SC_MINEIG_Y;
      sa.sap = SC_ALPHA_P;
      sa.sad = SC_ALPHA_D;
      sa.pdslot = SC_PDFEAS;
      alpha_fused = false;
    }
    update_state<T><<<RED_G, 256, 0, stream>>>(X, dX, Y, dY, nblk_el, x, dx, nx, cvec, y, dyv, n_y,
                                               bvec, sc + SC_ALPHA_P, sc + SC_ALPHA_D, info,
                                               info_count, upart, sa);
    if (world == 1 && !hasC) {  // the objectives from the partials, folded into one scalar launch
      zero_cy = true;
      fold(upart + RED_G, RED_G, 0, SC_DOT_CX);
      fold(upart + 2 * RED_G, RED_G, 0, SC_DOT_BY);
      scalars(prm, pd_feas, 3);
      zero_cy = false;
      return;
    }
    objectives(prm, pd_feas);
  }
  // <X,Y> partials of the current state, as update_state leaves them (after a state change
  // from the host: set_state, restore_state)
  void refresh_xy_part() {
    flat_reduce<T><<<RED_G, 256, 0, stream>>>(X, Y, nullptr, nullptr, nblk_el, 0, upart);
    HIPCHK(hipGetLastError());
  }

  void stage(int s, const clrsdp_params* prm, int pd_feas) {
    switch (s) {
      case CLRSDP_STAGE_MU_R: st_mu_r(prm, pd_feas); break;
      case CLRSDP_STAGE_XINV: st_xinv(); break;
      case CLRSDP_STAGE_SCHUR: st_schur(); break;
      case CLRSDP_STAGE_FACTOR: st_factor(); break;
      case CLRSDP_STAGE_RESIDUALS: st_residuals(true); break;
      case CLRSDP_STAGE_PREDICTOR: st_direction(4); break;
      case CLRSDP_STAGE_CORRECTOR_R: st_corrector_r(prm, pd_feas); break;
      case CLRSDP_STAGE_CORRECTOR: st_direction(6); break;
      case CLRSDP_STAGE_STEP: st_step(prm, pd_feas); break;
      case CLRSDP_STAGE_UPDATE: st_update(prm, pd_feas); break;
      default: throw ClrsdpError{CLRSDP_E_ARG, "bad stage"};
    }
    HIPCHK(hipGetLastError());
  }

  // both parse the host mirror filled by stat_fetch().  Failure bits: 1 S_j, 2 Q, 4 X
  // (Cholesky), 8 X^-1 by LU, 16 Y (step length); with world > 1 the OR over all ranks
  // (info_G, STEP's exchange), so every rank returns the same code
  int fail_bits(const int* h) const {
    int b = 0;
    for (int i = 0; i < nb(); ++i) {
      if (h[i]) b |= 4;
      if (h[info_Y0 + i]) b |= 16;
      if (h[info_L0 + i]) b |= 8;
    }
    for (int i = 0; i < nc() + nc2; ++i)
      if (h[info_S0 + i]) b |= 1;
    if (h[info_Q0]) b |= 2;
    return b;
  }
  int check_info(const char* blk = nullptr) {
    const int* h = reinterpret_cast<const int*>((blk ? blk : stat_host) + stat_info_off);
    // local bits always (run_stage reports a failure at the stage where it happens); with
    // world > 1 also the OR over all ranks, which STEP's exchange wrote into info_G
    const int b = fail_bits(h) | ((world > 1 && (comm || xfn)) ? h[info_G] : 0);
    if (b & 4) {
      if (lu_x()) {  // X^-1 came from LU; cho!(X) of the step length failed (MPMP.jl:1846-1882)
        err = "The step length could not be calculated correctly (X not PD).";
        return CLRSDP_E_STEP;
      }
      err = "X block not positive definite (spd_inv! failed)";
      return CLRSDP_E_NOT_PD_X;
    }
    if (b & 8) { err = "The inverse was not computed correctly. Try again with higher precision"; return CLRSDP_E_NOT_PD_X; }
    if (b & 1) { err = "S was not decomposed succesfully, try again with higher precision"; return CLRSDP_E_NOT_PD_S; }
    if (b & 2) { err = "Q was not decomposed correctly. Try restarting with a higher precision."; return CLRSDP_E_NOT_PD_Q; }
    if (b & 16) { err = "The step length could not be calculated correctly (Y not PD)."; return CLRSDP_E_STEP; }
    return CLRSDP_OK;
  }
  // A Cholesky failure the LU fallback covers: switch (for the rest of the solve) and report
  // true, so the caller re-runs the loop body (its update was skipped, the state is unchanged)
  bool fallback(int rc) {
    if (!(fact_flags & CLRSDP_FACT_FALLBACK)) return false;
    int add = 0;
    if ((rc == CLRSDP_E_NOT_PD_S || rc == CLRSDP_E_NOT_PD_Q) && !lu_sq()) add = CLRSDP_FACT_LU_SQ;
    else if (rc == CLRSDP_E_NOT_PD_X && !lu_x()) add = CLRSDP_FACT_LU_X;
    if (!add || !lu_fits()) return false;  // beyond the LU panel: the reference's error stands
    build_lu_plans();
    fact_flags |= add;
    drop_graphs();
    ++fallbacks;
    return true;
  }
  int fallbacks = 0;

  void read_stats(clrsdp_iter_stats* st, const char* blk = nullptr) {
    const T* h = reinterpret_cast<const T*>(blk ? blk : stat_host);
    auto f = [&](int i) { return Num<T>::hi(h[i]); };
    st->mu = f(SC_MU);
    st->P_err = f(SC_ERR_PMAT);
    st->p_err = f(SC_ERR_PVEC);
    st->d_err = f(SC_ERR_DVEC);
    st->alpha_p = f(SC_ALPHA_P);
    st->alpha_d = f(SC_ALPHA_D);
    st->beta_c = f(SC_BETA_C);
    st->p_obj = f(SC_POBJ);
    st->d_obj = f(SC_DOBJ);
    auto limbs_of = [&](int i, double* dst) {
      const double* l = reinterpret_cast<const double*>(&h[i]);
      for (int q = 0; q < 4; ++q) dst[q] = q < Num<T>::W ? l[q] : 0.0;
    };
    limbs_of(SC_GAP, st->gap_w);
    limbs_of(SC_ERR_PMAT, st->P_err_w);
    limbs_of(SC_ERR_PVEC, st->p_err_w);
    limbs_of(SC_ERR_DVEC, st->d_err_w);
  }

  int initial(const clrsdp_params* prm, clrsdp_iter_stats* st) override {
    if (!uploaded) { err = "constraints not uploaded"; return CLRSDP_E_STATE; }
    std::memset(st, 0, sizeof(*st));
    st_residuals(false);
    objectives(prm, 0, 4);   // + gap / pd_feas / terminate of the initial point (device control)
    stat_fetch();
    read_stats(st);
    return CLRSDP_OK;
  }

  // Enqueue one loop body (all stages) on `stream`, with the side stream joined back in.
  void enqueue_iteration(const clrsdp_params* prm, int pd_feas) {
    segs.clear();
    // (the status words are cleared by the first scalar launch of MU_R)
    auto mark = [&](int s) {
      if (timing == 1) HIPCHK(hipEventRecord(ev[s], stream));
    };
    // pipelined loop: P, p, d of every body that runs are copied aside (guarded by the halt
    // word), so a skipped body leaves the residuals of the last iteration that ran, which the
    // reference returns (MPMP.jl:1014-1024)
    const bool keep_res = pd_feas < 0;
    // The side stream runs everything of RESIDUALS and of the predictor's right-hand side that
    // does not need the Schur factorisation, as soon as its inputs exist, so that it overlaps
    // XINV, SCHUR and FACTOR (whose on-chip factorisations leave most CUs idle):
    //   after MU_R:  P = sum x_i A_i - X - C                      (state only)
    //   after SCHUR: d, the p-slabs, the maxima (A_Y from SCHUR); Z = X^-1 (P Y - R), U = Z V
    //                and rhs = -d - Tr(A_* Z)                     (the predictor's trace_A)
    //   after FACTOR's Q sum: chol(Q) -> L_Q^-1, Q^-1
    const hipStream_t main_s = stream;
    auto side = [&](hipEvent_t ev, auto&& work) {
      HIPCHK(hipEventRecord(ev, main_s));
      HIPCHK(hipStreamWaitEvent(aux, ev, 0));
      StreamSwitch on_aux(stream, aux);
      work();
    };
    static const bool fr = !env_off("CLRSDP_FUSE_R");
    fuse_r = fr && std::is_same<T, double>::value && timing != 1 && !p_xir.h.empty();
    mark(CLRSDP_STAGE_MU_R);
    stage(CLRSDP_STAGE_MU_R, prm, pd_feas);
    // V^T Y of the Schur stage only needs the state: it runs beside chol_inv(X, Y), which leaves
    // half the CUs idle, and SCHUR waits for it (ev_ty) before the pairs launch
    const bool ty_side = fast_schur && !p_ty.h.empty() && exp_knob != 4 && !(schur_fused && fused_y);
    // P = sum x_i A_i - X - C is first read by the side stream's Z after SCHUR: enqueued there
    // (one fork of the critical path fewer) unless V^T Y needs the fork anyway
    // (CLRSDP_P_AT_SCHUR=0: beside chol_inv(X, Y) as before)
    static const bool p_at_schur = !env_off("CLRSDP_P_AT_SCHUR");
    const bool p_late = p_at_schur && !ty_side;
    if (!p_late)
      side(ev_m, [&] {
        if (ty_side) {
          p_ty.launch(stream, 1.0, 0.0);
          HIPCHK(hipEventRecord(ev_ty, stream));
          ty_ahead = true;
        }
        residuals_P();
      });
    mark(CLRSDP_STAGE_XINV);
    stage(CLRSDP_STAGE_XINV, prm, pd_feas);
    fuse_r = false;
    mark(CLRSDP_STAGE_SCHUR);
    stage(CLRSDP_STAGE_SCHUR, prm, pd_feas);
    // (Z waits for SCHUR although it could start after XINV: beside the MFMA-bound Schur
    // products it only slowed them down, beside FACTOR's latency-bound factorisations it is free)
    // The predictor's Z first (its MFMA chain fills the CUs that chol(S11) leaves idle), then the
    // residuals; the right-hand side (U = Z V and its column sums) after FACTOR's side products
    // W1^T W1 and B2' (ev_w), which are on the critical path to W2 = L22^-1 B2'
    side(ev_s, [&] {
      if (p_late) residuals_P();
      direction_Z();
      residuals_rest(true);
      if (keep_res) {
        copy_guarded2(Pres, P, nblk_el, dres, dvec, nx);
      }
    });
    mark(CLRSDP_STAGE_FACTOR);
    factor_local(true);
    {
      if (w_split) HIPCHK(hipStreamWaitEvent(aux, ev_w, 0));
      StreamSwitch on_aux(stream, aux);
      direction_rhs();
      HIPCHK(hipEventRecord(ev_r, aux));
    }
    // side stream: chol(Q) -> L_Q^-1, waited for just before the first Q solve
    HIPCHK(hipEventRecord(ev_qa, main_s));
    HIPCHK(hipStreamWaitEvent(aux, ev_qa, 0));
    {
      StreamSwitch on_aux(stream, aux);
      factor_q();
    }
    HIPCHK(hipEventRecord(ev_q, aux));
    pending_q = true;
    if (capturing && inject_capture_fail)
      throw ClrsdpError{CLRSDP_E_HIP, "injected capture failure (CLRSDP_INJECT_CAPTURE_FAIL)"};
    mark(CLRSDP_STAGE_RESIDUALS);
    HIPCHK(hipStreamWaitEvent(main_s, ev_r, 0));
    static const bool defer_res = !env_off("CLRSDP_DEFER_RES");  // (round 6; =0 for A/B)
    residuals_finish(defer_res && timing != 1);
    if (keep_res) copy_guarded(pres, pvec, n_y);
    HIPCHK(hipGetLastError());
    mark(CLRSDP_STAGE_PREDICTOR);
    direction_rest(4);   // Z, U and rhs came from the side stream
    // (STEP's alpha is formed inside UPDATE's launch; CLRSDP_FUSE_ALPHA=0 keeps the scalar
    // launch; the per-stage timing mode keeps it so STEP's time includes alpha)
    static const bool fa = !env_off("CLRSDP_FUSE_ALPHA");
    fuse_alpha = fa && timing != 1;
    xy_ov_body = timing != 1;
    for (int s = CLRSDP_STAGE_CORRECTOR_R; s < CLRSDP_NUM_STAGES; ++s) {
      mark(s);
      stage(s, prm, pd_feas);
    }
    fuse_alpha = false;
    xy_ov_body = false;
    if (xy_ov) {  // (STEP did not run: join the side stream anyway)
      HIPCHK(hipStreamWaitEvent(stream, ev_stx, 0));
      xy_ov = false;
    }
    if (pending_q) {
      HIPCHK(hipStreamWaitEvent(stream, ev_q, 0));
      pending_q = false;
    }
    if (pending_x21) {
      HIPCHK(hipStreamWaitEvent(stream, ev_x21, 0));
      pending_x21 = false;
    }
    if (pending_sinv) {
      HIPCHK(hipStreamWaitEvent(stream, ev_sinv, 0));
      pending_sinv = false;
    }
    if (timing == 1) HIPCHK(hipEventRecord(ev[CLRSDP_NUM_STAGES], stream));
  }

  // One hipGraph per pd_feas value replays the whole loop body with a single launch (one
  // process per GPU with no exchange, and no per-stage timing).  The scalar parameters are
  // baked into the graph, so a change of them re-captures.
  // pd_feas 0, 1 and decided on the device (two instances of that one, used alternately, so a
  // launch never waits for the previous launch of the same executable graph)
  hipGraphExec_t gexec[4] = {nullptr, nullptr, nullptr, nullptr};
  clrsdp_params gprm[4];
  unsigned graph_launches = 0;
  // multi-word bodies are enqueued eagerly by default: C5 (qd) 719-730 against 672-706 it/s,
  // C4 (dd) 620-625 against 600-617 with the replayed graph (A/B, round 4); fp64 keeps the
  // replay (C3 equal, C2 2288-2315 against 2122-2288 eager); CLRSDP_GRAPH_MW=1 replays
  // multi-word bodies too
  bool use_graph = !env_on("CLRSDP_NO_GRAPH") && (sizeof(T) == 8 || env_on("CLRSDP_GRAPH_MW"));
  // multi-rank loop bodies with the native communicator are enqueued eagerly by default (the
  // pipelined host loop hides the enqueue); CLRSDP_GRAPH_RCCL=1 captures the all-gathers into
  // the replayed graph as well
  bool graph_rccl = env_on("CLRSDP_GRAPH_RCCL");
  void set_graph(int on) override {
    if (inflight) throw ClrsdpError{CLRSDP_E_STATE, "set_graph with loop bodies in flight"};
    use_graph = on != 0;
  }
  // the exchange the loop body uses: backend 0 none (one rank), 1 the native RCCL communicator
  // (nranks = ncclCommCount), 2 the registered callback (nranks = world_size)
  void comm_info(int* nranks, int* backend) const override {
    *backend = comm ? 1 : (xfn ? 2 : 0);
    *nranks = world;
    if (comm && rccl().comm_count) {
      int n = 0;
      if (rccl().comm_count(comm, &n) == ncclSuccess) *nranks = n;
    }
  }
  bool graph_ok() const { return use_graph && timing != 1 && (world == 1 || (comm && graph_rccl)); }
  // forget every captured loop body (they are re-captured on their next use)
  void drop_graphs() {
    for (hipGraphExec_t& g : gexec)
      if (g) {
        HIPCHK(hipGraphExecDestroy(g));
        g = nullptr;
      }
  }
  void launch_graph(const clrsdp_params* prm, int pd_feas) {
    // (one executable for every pipelined body measured the same as two alternating, round 4)
    const int g = pd_feas < 0 ? 2 + (graph_launches++ & 1) : (pd_feas ? 1 : 0);
    if (!gexec[g] || std::memcmp(&gprm[g], prm, sizeof(*prm)) != 0) {
      if (gexec[g]) HIPCHK(hipGraphExecDestroy(gexec[g]));
      gexec[g] = nullptr;
      hipGraph_t graph = nullptr;
      HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
      try {
        capturing = true;
        enqueue_iteration(prm, pd_feas);
        capturing = false;
      } catch (...) {
        capturing = false;
        // join the side stream (it may have been forked into the capture) so that the capture
        // ends cleanly and the streams stay usable
        if (aux != stream && hipEventRecord(ev_join, aux) == hipSuccess)
          (void)hipStreamWaitEvent(stream, ev_join, 0);
        if (aux2 != stream && hipEventRecord(ev_join2, aux2) == hipSuccess)
          (void)hipStreamWaitEvent(stream, ev_join2, 0);
        (void)hipStreamEndCapture(stream, &graph);
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipGetLastError();
        throw;
      }
      HIPCHK(hipStreamEndCapture(stream, &graph));
      HIPCHK(hipGraphInstantiate(&gexec[g], graph, nullptr, nullptr, 0));
      HIPCHK(hipGraphDestroy(graph));
      gprm[g] = *prm;
    }
    HIPCHK(hipGraphLaunch(gexec[g], stream));
  }

  // A sharded body whose capture fails (CLRSDP_GRAPH_RCCL with an RCCL that cannot be captured)
  // is enqueued eagerly instead, and the handle stays eager from then on; one rank rethrows (its
  // capture has no collective in it, so a failure there is a real error)
  // CLRSDP_INJECT_CAPTURE_FAIL=1 (tests only, read per handle): the first capture of a loop body
  // throws half-way through its enqueue, after the side streams were forked and the pending
  // flags set, and the body takes the sharded path's eager fallback even at one rank
  bool inject_capture_fail = env_on("CLRSDP_INJECT_CAPTURE_FAIL");
  bool capturing = false;
  // the per-body enqueue state a failed (partial) capture may have left set; an eager re-enqueue
  // must not wait on events recorded only inside the aborted capture
  void reset_body_state() {
    pending_q = pending_x21 = pending_sinv = false;
    ty_ahead = false;
    w_split = false;
    dy_dot_ready = false;
    alpha_fused = false;
    fuse_alpha = false;
    fuse_r = false;
    xy_ov_body = xy_ov = false;
  }
  void launch_graph_or_eager(const clrsdp_params* prm, int pd_feas) {
    if (world == 1 && !inject_capture_fail) {
      launch_graph(prm, pd_feas);
      return;
    }
    try {
      launch_graph(prm, pd_feas);
    } catch (const ClrsdpError& e) {
      std::fprintf(stderr, "clrsdp: graph capture of the sharded loop body failed (%s); "
                           "enqueueing it eagerly from now on\n", e.msg.c_str());
      graph_rccl = false;
      inject_capture_fail = false;
      reset_body_state();
      enqueue_iteration(prm, pd_feas);
    }
  }
  int iterate(const clrsdp_params* prm, int pd_feas, clrsdp_iter_stats* st) override {
    if (!uploaded) { err = "constraints not uploaded"; return CLRSDP_E_STATE; }
    if (inflight) { err = "iterate with loop bodies in flight (call iterate_wait)"; return CLRSDP_E_STATE; }
    for (;;) {
      const int rc = iterate_once(prm, pd_feas, st);
      if (!fallback(rc)) return rc;
    }
  }
  int iterate_once(const clrsdp_params* prm, int pd_feas, clrsdp_iter_stats* st) {
    if (graph_ok()) launch_graph_or_eager(prm, pd_feas);
    else enqueue_iteration(prm, pd_feas);
    res_from_copy = false;
    std::memset(st, 0, sizeof(*st));
    stat_fetch();
    read_stats(st);
    if (timing == 2) {  // the SCHUR stage of the body that just ran (device clock stamps)
      const unsigned long long* t = reinterpret_cast<const unsigned long long*>(stat_host + stat_stamp_off);
      // the durations of its three launches (V^T X^-1, V^T Y -- ahead on the side stream in a
      // loop body -- and the pairs), first workgroup start to last workgroup end each
      double ticks = 0.0;
      for (int q = 0; q < 3; ++q)
        if (t[2 * q + 1] > t[2 * q]) ticks += (double)(t[2 * q + 1] - t[2 * q]);
      st->phase_ms[CLRSDP_STAGE_SCHUR] = ticks * 1e-5;  // 100 MHz
    }
    if (timing == 1) {
      for (int s = 0; s < CLRSDP_NUM_STAGES; ++s) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ev[s], ev[s + 1]));
        st->phase_ms[s] = ms;
      }
      for (const auto& g : segs) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, seg_pool[g[1]], seg_pool[g[2]]));
        st->inner_ms[g[0]] += ms;
      }
      st->inner_ms[CLRSDP_INNER_SCHUR] = st->phase_ms[CLRSDP_STAGE_SCHUR];
    }
    const int rc = check_info();
    st->status = rc;
    return rc;
  }
  // 0: off (graph replay); 1: every stage between HIP events, no graph; 2: graph replay, and the
  // SCHUR stage timed inside the replayed body by the 100 MHz clock: the sum over its launches of
  // first workgroup start to last workgroup end (atomics in the stat block)
  void set_timing(int on) override {
    if (on < 0 || on > 2) throw ClrsdpError{CLRSDP_E_ARG, "timing mode must be 0, 1 or 2"};
    timing = on;
  }

  // device-side snapshot of the iterate (x, X, y, Y) and the scalar slots, stream-ordered
  T* snap = nullptr;
  bool snapped = false;
  void snap_copy(bool save) {
    const int64_t B = nblk_el;
    T* dst[5] = {snap, snap + nx, snap + nx + B, snap + nx + 2 * B, snap + nx + 2 * B + n_y};
    T* src[5] = {x, X, Y, y, sc};
    const int64_t cnt[5] = {nx, B, B, n_y, (int64_t)SC_COUNT};
    for (int i = 0; i < 5; ++i)
      if (cnt[i])
        HIPCHK(hipMemcpyAsync(save ? dst[i] : src[i], save ? src[i] : dst[i], cnt[i] * sizeof(T),
                              hipMemcpyDeviceToDevice, stream));
  }
  void save_state() override {
    if (!snap) snap = dmalloc<T>((size_t)nx + 2 * (size_t)nblk_el + (size_t)n_y + SC_COUNT);
    snap_copy(true);
    snapped = true;
  }
  void restore_state() override {
    dy_dot_ready = false;
    if (!snapped) throw ClrsdpError{CLRSDP_E_STATE, "restore_state without save_state"};
    snap_copy(false);
    refresh_xy_part();
  }

  // ---- pipelined loop: the host enqueues loop body k+1 before it reads the log row of body k.
  // pd_feas and terminate() are evaluated on the device at the end of each update (and by
  // initial_residuals); a body enqueued after the device decided to terminate changes no
  // state (the halt word guards every update like a failed factorisation) and reports ran = 0.
  char* ring_host[2] = {nullptr, nullptr};
  hipEvent_t ring_ev[2] = {nullptr, nullptr};
  int ring_head = 0, inflight = 0;
  clrsdp_params last_prm{};
  int iterate_async(const clrsdp_params* prm) override {
    if (!uploaded) { err = "constraints not uploaded"; return CLRSDP_E_STATE; }
    last_prm = *prm;
    if (inflight >= 2) { err = "two loop bodies already in flight (call iterate_wait)"; return CLRSDP_E_STATE; }
    if (!ring_host[0]) {
      for (int i = 0; i < 2; ++i) {
        HIPCHK(hipHostMalloc((void**)&ring_host[i], stat_bytes, hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&ring_ev[i], hipEventDisableTiming));
      }
    }
    if (graph_ok()) launch_graph_or_eager(prm, -1);
    else enqueue_iteration(prm, -1);
    const int slot = (ring_head + inflight) % 2;
    HIPCHK(hipMemcpyAsync(ring_host[slot], stat_dev, stat_bytes, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipEventRecord(ring_ev[slot], stream));
    ++inflight;
    return CLRSDP_OK;
  }
  int iterate_wait(clrsdp_iter_stats* st, int* ran) override {
    if (!inflight) { err = "no loop body in flight"; return CLRSDP_E_STATE; }
    const int slot = ring_head;
    ring_head = (ring_head + 1) % 2;
    --inflight;
    HIPCHK(hipEventSynchronize(ring_ev[slot]));
    std::memset(st, 0, sizeof(*st));
    read_stats(st, ring_host[slot]);
    const int* h = reinterpret_cast<const int*>(ring_host[slot] + stat_info_off);
    const bool halted = h[info_H] != 0;
    if (ran) *ran = halted ? 0 : 1;
    res_from_copy = true;
    if (halted) return CLRSDP_OK;   // skipped body: its factorisations may fail, nothing applied
    const int rc = check_info(ring_host[slot]);
    st->status = rc;
    const int behind = inflight;
    // a failed body: the bodies behind it may still execute (from the replayed graphs), so they
    // are waited for before fallback() destroys any graph
    if (rc != CLRSDP_OK)
      for (int q = 0; q < behind; ++q) HIPCHK(hipEventSynchronize(ring_ev[(ring_head + q) % 2]));
    if (fallback(rc)) {
      // the bodies behind this one ran on the same (unchanged) state and failed alike:
      // re-enqueue this body and those behind it with the LU factorisations
      inflight = 0;
      const clrsdp_params prm = last_prm;
      for (int q = 0; q <= behind; ++q) {
        const int r2 = iterate_async(&prm);
        if (r2) return r2;
      }
      return iterate_wait(st, ran);
    }
    return rc;
  }

  int run_stage(int s, const clrsdp_params* prm, int pd_feas) override {
    if (!uploaded) { err = "constraints not uploaded"; return CLRSDP_E_STATE; }
    if (s == 0) {
      HIPCHK(hipMemsetAsync(info, 0, info_count * sizeof(int), stream));
      segs.clear();
    }
    stage(s, prm, pd_feas);
    flush_scalars();
    stat_fetch();
    return check_info();
  }

  void get_buffer(int buf, double* host, int64_t* count) override {
    const T* src = nullptr;
    int64_t n = 0;
    switch (buf) {
      case CLRSDP_BUF_X: src = X; n = nblk_el; break;
      case CLRSDP_BUF_Y: src = Y; n = nblk_el; break;
      case CLRSDP_BUF_XINV: src = Xinv; n = nblk_el; break;
      case CLRSDP_BUF_R: src = R; n = nblk_el; break;
      case CLRSDP_BUF_S: src = S; n = nS; break;
      case CLRSDP_BUF_AY: src = AY; n = nAY; break;
      case CLRSDP_BUF_Q: src = Q; n = n_y * n_y; break;
      case CLRSDP_BUF_P: src = res_from_copy ? Pres : P; n = nblk_el; break;
      case CLRSDP_BUF_PVEC: src = res_from_copy ? pres : pvec; n = n_y; break;
      case CLRSDP_BUF_DVEC: src = res_from_copy ? dres : dvec; n = nx; break;
      case CLRSDP_BUF_DX: src = dx; n = nx; break;
      case CLRSDP_BUF_DXMAT: src = dX; n = nblk_el; break;
      case CLRSDP_BUF_DY: src = dyv; n = n_y; break;
      case CLRSDP_BUF_DYMAT: src = dY; n = nblk_el; break;
      case CLRSDP_BUF_XVEC: src = x; n = nx; break;
      case CLRSDP_BUF_YVEC: src = y; n = n_y; break;
      case CLRSDP_BUF_SCALARS: src = sc; n = SC_COUNT; break;
      default: throw ClrsdpError{CLRSDP_E_ARG, "bad buffer id"};
    }
    if (count) *count = n;
    if (host) get(src, host, n, 0, n);
    if (host && buf == CLRSDP_BUF_S && s_lower) {  // (fp64 only) the full symmetric S_j
      for (int c = 0; c < nc(); ++c) {
        const int64_t D = Ds[oc[c]];
        double* Sc = host + c_Soff[c];
        for (int64_t j = 0; j < D; ++j)
          for (int64_t i = 0; i < j; ++i) Sc[i + j * D] = Sc[j + i * D];
      }
    }
  }

  int64_t exchange_bytes() const override { return xcap * (int64_t)sizeof(T); }
  void set_exchange(clrsdp_exchange_fn fn, void* ctx, void* send, void* recv) override {
    if (comm) throw ClrsdpError{CLRSDP_E_STATE, "the handle exchanges over its own RCCL communicator"};
    xfn = fn;
    xctx = ctx;
    if (send && recv) {
      xsend = reinterpret_cast<T*>(send);
      xrecv = reinterpret_cast<T*>(recv);
    } else {
      xsend = xrecv = own_send;
    }
  }
  void comm_init(const uint8_t* id) override {
    if (comm) throw ClrsdpError{CLRSDP_E_STATE, "RCCL communicator already initialised"};
    if (inflight) throw ClrsdpError{CLRSDP_E_STATE, "loop bodies in flight"};
    ncclUniqueId uid;
    static_assert(sizeof(uid) == CLRSDP_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(&uid, id, sizeof(uid));
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamSynchronize(stream));
    if (world > 1 && !comm_recv) comm_recv = dmalloc<T>((size_t)world * xcap);
    ncclComm_t c = nullptr;
    RCCLCHK(rccl().comm_init_rank(&c, world, uid, rank));  // on failure the handle keeps no comm
    comm = c;
    xsend = own_send;
    xrecv = world > 1 ? comm_recv : own_send;
    // one eager all-gather of the full capacity: RCCL connects its channels on first use, which
    // must not happen inside a graph capture
    RCCLCHK(rccl().all_gather(xsend, xrecv, (size_t)(xcap * (int64_t)sizeof(T)), ncclUint8, comm,
                              stream));
    HIPCHK(hipStreamSynchronize(stream));
    // graphs captured before carry no all-gathers
    drop_graphs();
  }
  void set_stream(void* s) override { stream = s ? reinterpret_cast<hipStream_t>(s) : own_stream; }
  void* get_stream() const override { return (void*)stream; }
  void synchronize() override { HIPCHK(hipStreamSynchronize(stream)); }
};

// Stand-alone compute_step_length (MPMP.jl:1829-1898) of a block-diagonal pair (M, dM), fp64:
// the same kernels as STAGE_STEP (L^-1 on chip and two MFMA products for blocks <= 128, potrf +
// two triangular solves above), then lambda_min per block and alpha.
struct DevBuf {
  std::vector<void*> p;
  ~DevBuf() {
    for (void* q : p) (void)hipFree(q);
  }
  template <class X>
  X* alloc(size_t n) {
    X* q = dmalloc<X>(n);
    p.push_back(q);
    return q;
  }
};

// lambda_min of each symmetric block at the word type T (the eigenvalue part of
// compute_step_length, MPMP.jl:1857-1870): planes in, planes out
template <class T>
void eigmin_words(int device, int64_t nblk, const int64_t* n, const double* Ap, double* ep) {
  constexpr int W = Num<T>::W;
  DeviceGuard dg(device);
  std::vector<int64_t> off(nblk + 1, 0);
  for (int64_t b = 0; b < nblk; ++b) {
    if (n[b] <= 0 || n[b] > 4096) throw ClrsdpError{CLRSDP_E_ARG, "block size out of range"};
    off[b + 1] = off[b] + n[b] * n[b];
  }
  const int64_t tot = off[nblk];
  // planes -> interleaved limbs (the layout of T)
  std::vector<double> h((size_t)tot * W);
  for (int64_t e = 0; e < tot; ++e)
    for (int q = 0; q < W; ++q) h[(size_t)e * W + q] = Ap[(size_t)q * tot + e];
  DevBuf mem;
  T* A = mem.alloc<T>(tot);
  T* eig = mem.alloc<T>(nblk);
  HIPCHK(hipMemcpy(A, h.data(), (size_t)tot * sizeof(T), hipMemcpyHostToDevice));
  MatPlan<T> eg;
  for (int64_t b = 0; b < nblk; ++b) eg.add(A + off[b], (int)n[b], (int)n[b]);
  eg.finalize();
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{s};
  eg.eigmin(s, eig);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  std::vector<double> he((size_t)nblk * W);
  HIPCHK(hipMemcpy(he.data(), eig, (size_t)nblk * sizeof(T), hipMemcpyDeviceToHost));
  for (int64_t b = 0; b < nblk; ++b)
    for (int q = 0; q < W; ++q) ep[(size_t)q * nblk + b] = he[(size_t)b * W + q];
}

int step_length_f64(int device, int64_t nblk, const int64_t* n, const double* Mh, const double* dMh,
                    double gamma, double* alpha, double* min_eig, std::string& err) {
  DeviceGuard dg(device);
  std::vector<int64_t> off(nblk + 1, 0);
  int nmax = 0;
  for (int64_t b = 0; b < nblk; ++b) {
    if (n[b] <= 0 || n[b] > 4096) throw ClrsdpError{CLRSDP_E_ARG, "block size out of range"};
    off[b + 1] = off[b] + n[b] * n[b];
    nmax = std::max(nmax, (int)n[b]);
  }
  const int64_t tot = off[nblk];
  DevBuf mem;
  double* M = mem.alloc<double>(tot);
  double* dM = mem.alloc<double>(tot);
  double* L = mem.alloc<double>(tot);
  double* t1 = mem.alloc<double>(tot);
  double* t2 = mem.alloc<double>(tot);
  double* eig = mem.alloc<double>(nblk);
  int* info = mem.alloc<int>(nblk);
  HIPCHK(hipMemcpy(M, Mh, tot * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dM, dMh, tot * sizeof(double), hipMemcpyHostToDevice));
  CholInvPlan<double> ci;
  GemmPlan<double> g1, g2;
  g2.tb = true;
  g2.sym = true;  // exactly symmetric L^-1 dM L^-T (eigmin_reg reads only A(i, j))
  MatPlan<double> fac, eg;
  TrsmPlan<double> s1, s2;
  std::vector<BlkDesc> big;
  for (int64_t b = 0; b < nblk; ++b) {
    const int nb = (int)n[b];
    const int64_t o = off[b];
    if (nb <= 128) {
      ci.add(M + o, nb, nb, L + o, nb);                                    // L <- L_M^-1
      g1.add(L + o, nb, dM + o, nb, nullptr, nb, t1 + o, nb, nb, nb, nb);  // t1 = L^-1 dM
      g2.add(t1 + o, nb, L + o, nb, nullptr, nb, t2 + o, nb, nb, nb, nb);  // t2 = t1 L^-T
    } else {
      fac.add(L + o, nb, nb);          // L <- chol(M)
      s1.add(L + o, nb, t1 + o, nb, nb, nb);
      s2.add(L + o, nb, t2 + o, nb, nb, nb);
      big.push_back(BlkDesc{o, nb, 0});
    }
    eg.add(t2 + o, nb, nb);
  }
  ci.finalize(); g1.finalize(); g2.finalize(); fac.finalize(); eg.finalize();
  s1.finalize(); s2.finalize();
  PlanBase bd_owner;
  BlkDesc* d_big = big.empty() ? nullptr : bd_owner.own(big);
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{s};
  ci.launch(s, info);
  g1.launch(s, 1.0, 0.0);
  g2.launch(s, 1.0, 0.0);
  if (!big.empty()) {
    for (size_t q = 0; q < big.size(); ++q) {
      const int64_t o = big[q].off, nn = (int64_t)big[q].n * big[q].n;
      HIPCHK(hipMemcpyAsync(L + o, M + o, nn * sizeof(double), hipMemcpyDeviceToDevice, s));
      HIPCHK(hipMemcpyAsync(t1 + o, dM + o, nn * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    // the chol-inverse launch wrote info[0 .. #small); the potrf flags follow
    fac.potrf(s, info + ci.hin.size());
    s1.launch(s, false);                                             // t1 = L^-1 dM
    blk_sym2<double><<<dim3((unsigned)big.size(), 32), 128, 0, s>>>(d_big, t2, t1, 2);  // t2 = t1^T
    s2.launch(s, false);                                             // t2 = L^-1 dM^T L^-T
  }
  eg.eigmin(s, eig);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  std::vector<int> hinfo(nblk);
  std::vector<double> he(nblk);
  HIPCHK(hipMemcpy(hinfo.data(), info, nblk * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(he.data(), eig, nblk * sizeof(double), hipMemcpyDeviceToHost));
  for (int64_t b = 0; b < nblk; ++b)
    if (hinfo[b]) {
      err = "The step length could not be calculated correctly (M not positive definite).";
      return CLRSDP_E_STEP;
    }
  // the eigen kernels run in the (j,l) order of the plan: small blocks and large ones alike
  double mn = INFINITY;
  for (int64_t b = 0; b < nblk; ++b) {
    if (min_eig) min_eig[b] = he[b];
    mn = std::min(mn, he[b]);
  }
  *alpha = (mn > -gamma) ? 1.0 : -gamma / mn;  // MPMP.jl:1893-1897
  return CLRSDP_OK;
}

}  // namespace

struct clrsdp_handle {
  std::unique_ptr<HandleBase> impl;
};

#define GUARD(h, body)                                          \
  try {                                                         \
    DeviceGuard dg_(guard_dev(h));                              \
    body                                                        \
  } catch (const ClrsdpError& e) {                              \
    g_last_error = e.msg;                                       \
    if (h) (h)->impl->err = e.msg;                              \
    return e.code;                                              \
  } catch (const std::exception& e) {                           \
    g_last_error = e.what();                                    \
    if (h) (h)->impl->err = e.what();                           \
    return CLRSDP_E_HIP;                                        \
  }

static int guard_dev(const clrsdp_handle* h) {
  if (h) return h->impl->dev;
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

extern "C" {

int32_t clrsdp_version(void) { return 100; }

const char* clrsdp_last_error(const clrsdp_handle* h) {
  if (h && !h->impl->err.empty()) return h->impl->err.c_str();
  return g_last_error.c_str();
}

int32_t clrsdp_create(const clrsdp_desc* desc, const clrsdp_config* cfg, clrsdp_handle** out) {
  clrsdp_handle* h = nullptr;
  if (!desc || !cfg || !out) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, {
    DeviceGuard dg(cfg->device);
    auto* hh = new clrsdp_handle();
    if (cfg->precision_words == 1) hh->impl.reset(new Solver<double>(desc, cfg));
    else if (cfg->precision_words == 2) hh->impl.reset(new Solver<dd>(desc, cfg));
    else if (cfg->precision_words == 4) hh->impl.reset(new Solver<qd>(desc, cfg));
    else { delete hh; g_last_error = "precision_words must be 1, 2 or 4"; return CLRSDP_E_ARG; }
    *out = hh;
    return CLRSDP_OK;
  })
}

int32_t clrsdp_upload_constraints(clrsdp_handle* h, const double* V, const double* lambda,
                                  const double* B, const double* c, const double* b,
                                  const double* C) {
  if (!h || !V || !lambda || !B || !c || !b) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->upload(V, lambda, B, c, b, C); return CLRSDP_OK; })
}

int32_t clrsdp_set_state(clrsdp_handle* h, const double* x, const double* X, const double* y,
                         const double* Y) {
  if (!h || !x || !X || !y || !Y) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_state(x, X, y, Y); return CLRSDP_OK; })
}

int32_t clrsdp_get_state(clrsdp_handle* h, double* x, double* X, double* y, double* Y) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->get_state(x, X, y, Y); return CLRSDP_OK; })
}

int32_t clrsdp_initial_residuals(clrsdp_handle* h, const clrsdp_params* prm, clrsdp_iter_stats* st) {
  if (!h || !prm || !st) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { return h->impl->initial(prm, st); })
}

int32_t clrsdp_iterate(clrsdp_handle* h, const clrsdp_params* prm, int32_t pd_feas,
                       clrsdp_iter_stats* st) {
  if (!h || !prm || !st) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  if (pd_feas != 0 && pd_feas != 1) { g_last_error = "pd_feas must be 0 or 1"; return CLRSDP_E_ARG; }
  GUARD(h, { return h->impl->iterate(prm, pd_feas, st); })
}

int32_t clrsdp_set_control(clrsdp_handle* h, const clrsdp_control* ctl) {
  if (!h || !ctl) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_control(ctl); return CLRSDP_OK; })
}

int32_t clrsdp_iterate_async(clrsdp_handle* h, const clrsdp_params* prm) {
  if (!h || !prm) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { return h->impl->iterate_async(prm); })
}

int32_t clrsdp_iterate_wait(clrsdp_handle* h, clrsdp_iter_stats* st, int32_t* ran) {
  if (!h || !st) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, {
    int r = 0;
    const int rc = h->impl->iterate_wait(st, &r);
    if (ran) *ran = r;
    return rc;
  })
}

int32_t clrsdp_run_stage(clrsdp_handle* h, int32_t stage, const clrsdp_params* prm, int32_t pd_feas) {
  if (!h || !prm) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { return h->impl->run_stage(stage, prm, pd_feas); })
}

int32_t clrsdp_get_buffer(clrsdp_handle* h, int32_t buf, double* host, int64_t* count) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->get_buffer(buf, host, count); return CLRSDP_OK; })
}

int32_t clrsdp_exchange_bytes(const clrsdp_handle* h, int64_t* bytes) {
  if (!h || !bytes) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  *bytes = h->impl->exchange_bytes();
  return CLRSDP_OK;
}

int32_t clrsdp_set_exchange(clrsdp_handle* h, clrsdp_exchange_fn fn, void* ctx, void* send_dev,
                            void* recv_dev) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_exchange(fn, ctx, send_dev, recv_dev); return CLRSDP_OK; })
}

int32_t clrsdp_comm_unique_id(uint8_t* id) {
  if (!id) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  try {
    ncclUniqueId uid;
    RCCLCHK(rccl().get_unique_id(&uid));
    std::memcpy(id, &uid, sizeof(uid));
    return CLRSDP_OK;
  } catch (const ClrsdpError& e) {
    g_last_error = e.msg;
    return e.code;
  }
}

int32_t clrsdp_comm_init(clrsdp_handle* h, const uint8_t* id) {
  if (!h || !id) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->comm_init(id); return CLRSDP_OK; })
}

int32_t clrsdp_set_stream(clrsdp_handle* h, void* stream) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_stream(stream); return CLRSDP_OK; })
}

void* clrsdp_get_stream(const clrsdp_handle* h) { return h ? h->impl->get_stream() : nullptr; }

int32_t clrsdp_synchronize(clrsdp_handle* h) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->synchronize(); return CLRSDP_OK; })
}

int32_t clrsdp_save_state(clrsdp_handle* h) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->save_state(); return CLRSDP_OK; })
}

int32_t clrsdp_restore_state(clrsdp_handle* h) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->restore_state(); return CLRSDP_OK; })
}

int32_t clrsdp_step_length(int32_t device, int64_t nblocks, const int64_t* n, const double* M,
                           const double* dM, double gamma, double* alpha, double* min_eig) {
  if (nblocks <= 0 || !n || !M || !dM || !alpha) { g_last_error = "null argument or no blocks"; return CLRSDP_E_ARG; }
  try {
    std::string err;
    const int rc = step_length_f64(device, nblocks, n, M, dM, gamma, alpha, min_eig, err);
    if (rc) g_last_error = err;
    return rc;
  } catch (const ClrsdpError& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return CLRSDP_E_HIP;
  }
}

int32_t clrsdp_eigmin(int32_t device, int32_t words, int64_t nblocks, const int64_t* n,
                      const double* A, double* min_eig) {
  if (nblocks <= 0 || !n || !A || !min_eig) { g_last_error = "null argument or no blocks"; return CLRSDP_E_ARG; }
  try {
    if (words == 1) eigmin_words<double>(device, nblocks, n, A, min_eig);
    else if (words == 2) eigmin_words<mw::dd>(device, nblocks, n, A, min_eig);
    else if (words == 4) eigmin_words<mw::qd>(device, nblocks, n, A, min_eig);
    else { g_last_error = "words must be 1, 2 or 4"; return CLRSDP_E_ARG; }
    return CLRSDP_OK;
  } catch (const ClrsdpError& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return CLRSDP_E_HIP;
  }
}

int32_t clrsdp_set_timing(clrsdp_handle* h, int32_t on) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_timing(on); return CLRSDP_OK; })
}

int32_t clrsdp_set_graph(clrsdp_handle* h, int32_t on) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_graph(on); return CLRSDP_OK; })
}

int32_t clrsdp_comm_info(const clrsdp_handle* h, int32_t* nranks, int32_t* backend) {
  if (!h || !nranks || !backend) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  int n = 0, b = 0;
  h->impl->comm_info(&n, &b);
  *nranks = n;
  *backend = b;
  return CLRSDP_OK;
}

int32_t clrsdp_set_factorization(clrsdp_handle* h, int32_t flags) {
  if (!h) { g_last_error = "null handle"; return CLRSDP_E_ARG; }
  GUARD(h, { h->impl->set_factorization(flags); return CLRSDP_OK; })
}

int32_t clrsdp_get_factorization(const clrsdp_handle* h, int32_t* flags) {
  if (!h || !flags) { g_last_error = "null argument"; return CLRSDP_E_ARG; }
  *flags = h->impl->get_factorization();
  return CLRSDP_OK;
}

int32_t clrsdp_destroy(clrsdp_handle* h) {
  if (!h) return CLRSDP_OK;
  // CLRSDP_EIGMX_STATS=1: how many blocks eigmin_mx handed to the multi-word path so far (all
  // handles of the process; diagnostics only)
  if (env_on("CLRSDP_EIGMX_STATS")) {
    unsigned int fb = 0;
    if (hipMemcpyFromSymbol(&fb, HIP_SYMBOL(g_eigmx_fallbacks), sizeof(fb)) == hipSuccess)
      std::fprintf(stderr, "clrsdp: eigmin_mx multi-word fallbacks so far: %u\n", fb);
    std::vector<double> z(256 * 24);
    if (hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(g_eigmx_dbg), z.size() * sizeof(double)) == hipSuccess)
      for (int b = 0; b < 64; ++b) {
        const double* q = &z[b * 24];
        if (q[20] == 0.0 && q[23] == 0.0) continue;
        std::fprintf(stderr, "  block %d (last launch): eta %.2e %.2e %.2e %.2e lam %.17g lam2 %.17g rho %.17g temple %.2e\n",
                     b, q[16], q[17], q[18], q[19], q[20], q[21], q[22], q[23]);
      }
  }
  GUARD(h, { delete h; return CLRSDP_OK; })
}

}  // extern "C"
