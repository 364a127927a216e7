// Plain fp32 pointwise GEMMs on hipBLASLt, the library GEMM, with its fused
// bias (+ clamp(0, 6)) epilogue and the residual as C (beta = 1).  The fused
// kernels of mbv2_f32.hip stay hand-written; this only takes the plain
// [M][K] x [N][K]^T products where the library's fp32 MFMA GEMM beats the
// engine's 128 x 64 tile (profiles/r4_gemm_f32_vs_hipblaslt.txt: 113-128 vs
// 98-107 TF/s at K >= 256).  No workspace: every call is capture-safe and
// needs no allocation.  The library is the copy PyTorch already loaded (its
// symbols are bound at run time, so the process never holds two hipBLASLt
// builds: the ROCm one and torch's bundled one share a soname).
#include <dlfcn.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "kernels/mbv2.h"

namespace nnsx {
namespace kernels {

namespace {

// the hipBLASLt entry points used here, from the loaded library
struct Api {
  decltype(&hipblasLtCreate) create = nullptr;
  decltype(&hipblasLtMatmulDescCreate) desc_create = nullptr;
  decltype(&hipblasLtMatmulDescSetAttribute) desc_set = nullptr;
  decltype(&hipblasLtMatrixLayoutCreate) layout_create = nullptr;
  decltype(&hipblasLtMatmulPreferenceCreate) pref_create = nullptr;
  decltype(&hipblasLtMatmulPreferenceSetAttribute) pref_set = nullptr;
  decltype(&hipblasLtMatmulPreferenceDestroy) pref_destroy = nullptr;
  decltype(&hipblasLtMatmulAlgoGetHeuristic) heuristic = nullptr;
  decltype(&hipblasLtMatmul) matmul = nullptr;
  bool ok = false;
};

const Api& api() {
  static const Api a = [] {
    Api r;
    void* lib = nullptr;
    for (const char* n : {"libhipblaslt.so.1", "libhipblaslt.so"})
      if (!lib) lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);  // torch's copy, already mapped
    if (!lib) lib = dlopen("libhipblaslt.so.1", RTLD_NOW);
    if (!lib) return r;
    auto sym = [lib](auto& f, const char* name) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(lib, name)); };
    sym(r.create, "hipblasLtCreate");
    sym(r.desc_create, "hipblasLtMatmulDescCreate");
    sym(r.desc_set, "hipblasLtMatmulDescSetAttribute");
    sym(r.layout_create, "hipblasLtMatrixLayoutCreate");
    sym(r.pref_create, "hipblasLtMatmulPreferenceCreate");
    sym(r.pref_set, "hipblasLtMatmulPreferenceSetAttribute");
    sym(r.pref_destroy, "hipblasLtMatmulPreferenceDestroy");
    sym(r.heuristic, "hipblasLtMatmulAlgoGetHeuristic");
    sym(r.matmul, "hipblasLtMatmul");
    r.ok = r.create && r.desc_create && r.desc_set && r.layout_create && r.pref_create && r.pref_set &&
           r.pref_destroy && r.heuristic && r.matmul;
    return r;
  }();
  return a;
}

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};

// dev, M, N, K, Kpad, act, residual, bias: one plan per layer, so no descriptor
// is ever changed after it was built (calls from several threads share them)
using Key = std::tuple<int, int, int, int, int, int, int, const float*>;

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<Key, Plan> g_plans;

hipblasLtHandle_t handle(int dev) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  if (!api().ok || api().create(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
  g_handles[dev] = h;
  return h;
}

Plan make_plan(hipblasLtHandle_t h, int M, int N, int K, int Kpad, int act, const float* bias) {
  Plan p;
  // column-major view: D (N x M, ld N) = op(A) (N x K) . B (K x M) [+ C];
  // A = the weights [Npad][Kpad] row-major = Kpad x Npad column-major, transposed
  if (api().desc_create(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const hipblasLtEpilogue_t epi = act == 1 ? HIPBLASLT_EPILOGUE_CLAMP_BIAS_EXT : HIPBLASLT_EPILOGUE_BIAS;
  if (api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)) != HIPBLAS_STATUS_SUCCESS) return p;
  const hipDataType bt = HIP_R_32F;
  api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  if (api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) != HIPBLAS_STATUS_SUCCESS) return p;
  if (act == 1) {
    const float lo = 0.f, hi = 6.f;
    api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_ACT_ARG0_EXT, &lo, sizeof(lo));
    api().desc_set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_ACT_ARG1_EXT, &hi, sizeof(hi));
  }
  if (api().layout_create(&p.a, HIP_R_32F, K, N, Kpad) != HIPBLAS_STATUS_SUCCESS ||
      api().layout_create(&p.b, HIP_R_32F, K, M, K) != HIPBLAS_STATUS_SUCCESS ||
      api().layout_create(&p.c, HIP_R_32F, N, M, N) != HIPBLAS_STATUS_SUCCESS)
    return p;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (api().pref_create(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
  const uint64_t ws = 0;
  api().pref_set(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[4];
  int n = 0;
  const hipblasStatus_t st = api().heuristic(h, p.desc, p.a, p.b, p.c, p.c, pref, 4, res, &n);
  api().pref_destroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS || res[0].workspaceSize != 0)
    return p;
  p.algo = res[0].algo;
  p.ok = true;
  return p;
}

}  // namespace

// Opt-in (NNSX_F32_BLASLT=1, read at every call: GEMMs are issued at capture /
// eager time, never per graph replay).  Two pipeline shapes this path had not
// run before left the device with a memory-access fault -- PoseNet's 270k-row
// products and DeepLab's batch-16 17k-row products with the residual as C --
// while every shape of its tests and of the MobileNetV2 / SSD / DeepLab b8, b32
// runs was exact; until the library's failing configuration is pinned down the
// engine's own GEMM is the default (profiles/r4_blaslt_ab.txt: 0.6-3.8 % slower).
bool blaslt_enabled() {
  const char* e = std::getenv("NNSX_F32_BLASLT");
  return e && e[0] == '1';
}

bool blaslt_gemm_f32(const float* x, const float* wt, const float* bias, const float* res, float* y, int M, int N, int K,
                     int Kpad, int act, hipStream_t s) {
  if (act != 0 && act != 1) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const Plan* p = nullptr;
  hipblasLtHandle_t h = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    h = handle(dev);
    if (!h) return false;
    const Key key{dev, M, N, K, Kpad, act, res != nullptr, bias};
    auto it = g_plans.find(key);
    if (it == g_plans.end()) it = g_plans.emplace(key, make_plan(h, M, N, K, Kpad, act, bias)).first;
    p = &it->second;
  }
  if (!p->ok) return false;
  const float alpha = 1.f, beta = res ? 1.f : 0.f;
  const void* cptr = res ? static_cast<const void*>(res) : static_cast<const void*>(y);
  return api().matmul(h, p->desc, &alpha, wt, p->a, x, p->b, &beta, cptr, p->c, y, p->c, &p->algo, nullptr, 0, s) ==
         HIPBLAS_STATUS_SUCCESS;
}

}  // namespace kernels
}  // namespace nnsx
