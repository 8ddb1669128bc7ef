// pybind11 module `_dtf_hip`: thin launch entry points for the HIP kernels.
// Arguments are raw device addresses (tensor.data_ptr()) and the hipStream_t of the caller's
// current torch stream, so every launch is ordered on torch's stream (and captured into a
// hipGraph when torch is capturing).  Shape validation lives in distributedtensorflow_amd/ops/native.py;
// the launchers re-check the invariants their kernels index with.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"

namespace py = pybind11;

#define DTF_MAX_TAPS 64
struct TapTable { int n; int dh[DTF_MAX_TAPS]; int dw[DTF_MAX_TAPS]; };
struct TapTableW { int n; int dh[DTF_MAX_TAPS]; int dw[DTF_MAX_TAPS]; };
struct ConvGeom {
  int N, H, W, C, P, Q, sh, sw, Kout, Kpad, Ho, Wo, osh, osw, oh0, ow0, acc;
  const bf16_t* acc_src;
  const uint8_t* acc_mask;
  const float* bias;
  int relu;
  int nt;
  const float* lsc;
  const float* lsh;
  bf16_t* ly;
};
struct BnBwdEpi {
  const bf16_t* x; const float* mean; const float* invstd; const float* fsc; const float* fsh;
  const uint8_t* mask; float* part; int mkind; int row0;
};
constexpr int kWtMaxJobs = 48;
struct WtJobs {
  const bf16_t* src[kWtMaxJobs];
  bf16_t* dst[kWtMaxJobs];
  int K[kWtMaxJobs], T[kWtMaxJobs], C[kWtMaxJobs];
  int tile_end[kWtMaxJobs];
  int n;
};
void dtf_filter_transpose(const WtJobs&, hipStream_t);
struct WgradGeom { int N, H, W, C, P, Q, sh, sw, Kout, ldw; long m_per_split; long slab; };

// ---- launchers defined in the .hip translation units
int dtf_bn_partial_blocks(long M, int C);
long dtf_bn_workspace_floats(long M, int C);
void dtf_bn_fwd_stats(const bf16_t*, long, int, float*, hipStream_t);
void dtf_bn_fwd_finalize(const float*, long, int, const float*, const float*, float*, float*,
                         float, float, float*, float*, float*, float*, hipStream_t);
void dtf_bn_fwd_finalize_g(const float*, int, long, int, const float*, const float*, float*,
                           float*, float, float, float*, float*, float*, float*, hipStream_t);
long dtf_bn_workspace_floats_g(int, int);
int dtf_conv_stats_rows(long, int, int, int, int);
void dtf_conv_set_halo(int);
int dtf_gemm_conv_part_images(int, int, int, int, int, int);
void dtf_gemm_set_pp2_strided(int);
int dtf_conv_tile_rows(const ConvGeom&, const TapTable&, int bnb);
bool dtf_conv_bnl_ok(const ConvGeom&, const TapTable&);
void dtf_conv_set_bnl_probe(int);
void dtf_gemm_stream_set_bnb_probe(int);
void dtf_conv_set_halo_bnb(int);
void dtf_conv_set_dma_mode(int);
void dtf_conv_set_small_k(int);
void dtf_conv_set_stem_halo(int);
void dtf_conv_set_halo_strips(int);
void dtf_conv_set_halo_freg(int);
void dtf_bn_infer_finalize(int, const float*, const float*, const float*, const float*, float,
                           float*, float*, float*, float*, hipStream_t);
void dtf_bn_apply(const bf16_t*, const bf16_t*, bf16_t*, uint8_t*, const float*, const float*,
                  long, int, int, hipStream_t);
void dtf_bn_bwd_reduce(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*, const float*,
                       const float*, long, int, int, float*, const float*, const float*,
                       hipStream_t);
void dtf_bn_bwd_finalize_g(const float*, int, long, int, const float*, const float*, const float*,
                           float*, float*, float*, float*, float*, int, hipStream_t);
void dtf_bn_bwd_finalize(const float*, long, int, const float*, const float*, const float*,
                         float*, float*, float*, float*, float*, int, hipStream_t);
void dtf_relu_mask_apply(const bf16_t*, const uint8_t*, bf16_t*, long, hipStream_t);
void dtf_bn_apply_dual(const bf16_t*, const bf16_t*, bf16_t*, uint8_t*, const float*, const float*,
                       const float*, const float*, long, int, int, hipStream_t);
void dtf_bn_bwd_reduce_dual(const bf16_t*, const uint8_t*, const bf16_t*, const float*,
                            const float*, const bf16_t*, const float*, const float*, long, int,
                            float*, float*, hipStream_t);
void dtf_bn_bwd_apply_dual(const bf16_t*, const uint8_t*, const bf16_t*, const float*,
                           const float*, const float*, bf16_t*, const bf16_t*, const float*,
                           const float*, const float*, bf16_t*, long, int, hipStream_t);
void dtf_bn_bwd_apply(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*, const float*,
                      const float*, const float*, bf16_t*, bf16_t*, long, int, int, const float*,
                      const float*, hipStream_t);
void dtf_maxpool_fwd(const bf16_t*, bf16_t*, uint8_t*, int, int, int, int, int, int, int, int,
                     int, int, int, int, hipStream_t);
void dtf_maxpool_bwd(const bf16_t*, const uint8_t*, bf16_t*, int, int, int, int, int, int, int,
                     int, int, int, int, int, hipStream_t);
void dtf_gap_fwd(const bf16_t*, bf16_t*, int, int, int, hipStream_t);
void dtf_gap_bwd(const bf16_t*, bf16_t*, int, int, int, hipStream_t);
void dtf_bn_relu_maxpool_fwd(const bf16_t*, const float*, const float*, bf16_t*, uint8_t*, int,
                             int, int, int, int, int, int, int, int, int, int, int, hipStream_t);
void dtf_pool_set_blocked(int);
void dtf_s2d_set_rows(int);
int dtf_pool_bn_bwd_blocks(int, int, int, int);
void dtf_pool_bn_bwd_set_caps(int, int);
void dtf_pool_bn_bwd_reduce(const bf16_t*, const uint8_t*, const bf16_t*, const float*,
                            const float*, const float*, const float*, float*, int, int, int, int,
                            int, int, hipStream_t);
void dtf_pool_bn_bwd_apply(const bf16_t*, const uint8_t*, const bf16_t*, const float*,
                           const float*, const float*, const float*, const float*, bf16_t*, int,
                           int, int, int, int, int, hipStream_t);
void dtf_s2d_input(const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int,
                   hipStream_t);
void dtf_softmax_xent(const float*, const void*, int, int, int, float*, float*, float,
                      hipStream_t);
void dtf_sgd_momentum(float*, const float*, float*, bf16_t*, long, const float*, float, float,
                      float, int, int*, hipStream_t);
void dtf_adam(float*, const float*, float*, float*, bf16_t*, long, const float*, float, float,
              float, float, float, int*, hipStream_t);
void dtf_adagrad(float*, const float*, float*, bf16_t*, long, const float*, float, int*,
                 hipStream_t);
void dtf_lamb(float*, float*, float*, float*, bf16_t*, const void*, int, const float*,
              const float*, float, float, float, const float*, float, float*, int*, hipStream_t);
int dtf_lamb_chunk_bytes();
void dtf_sumsq(const float*, long, float*, hipStream_t);
void dtf_cast_f32_bf16(const float*, bf16_t*, long, hipStream_t);
void dtf_conv_igemm(const bf16_t*, const bf16_t*, bf16_t*, const ConvGeom&, const TapTable&, int,
                    float*, const BnBwdEpi&, hipStream_t);
bool dtf_conv_igemm_grouped(const bf16_t*, bf16_t*, const ConvGeom&, int, const bf16_t* const*,
                            const int*, const int*, const int*,
                            const std::vector<std::vector<int>>&,
                            const std::vector<std::vector<int>>&, const BnBwdEpi&, const int*,
                            hipStream_t);
void dtf_conv_wgrad(const bf16_t*, const bf16_t*, float*, float*, WgradGeom, const TapTableW&,
                    int, int, int, hipStream_t);

int dtf_conv_wgrad_splits(long, int, int, long, int);
int dtf_conv_wgrad_halo_splits(int, int, int, int, int, int, int, int, int, const TapTableW&);
void dtf_wgrad_set_halo(int);
void dtf_wgrad_set_stem(int);
int dtf_wgrad_stem_dz_splits(int);
void dtf_conv_wgrad_stem_dz(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*,
                            const float*, const float*, const float*, const float*, const float*,
                            float*, float*, int, int, hipStream_t);
void dtf_conv_set_halo_stages(int);
void dtf_wgrad_set_dma_mode(int);
void dtf_wgrad_set_pipe(int);
void dtf_wgrad_set_pp(int);
void dtf_wgrad_set_dense(int);
void dtf_wgrad_set_direct(int);
void dtf_wgrad_set_deep(int);
void dtf_conv_set_gemm(int);
void dtf_bn_set_nt(int);
void dtf_bn_set_grid_cap(int);
void dtf_bn_set_stats_blocks(int);
void dtf_conv_set_nt(int);
void dtf_gemm_set_nt(int);
void dtf_gemm_set_dbg(int);
void dtf_gemm_set_stream(int);
void dtf_gemm_stream_bnb(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int,
                         const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*,
                         const float*, const float*, const float*, const float*, const uint8_t*,
                         int, float*, int, hipStream_t, const bf16_t*, const bf16_t*, int);
bool dtf_gemm_stream_ok(int, int, int, int, int, int);
void dtf_gemm_stream_apply(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, const bf16_t*,
                           const float*, const float*, uint8_t*, hipStream_t);
void dtf_gemm_stream_bnb_dual(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int,
                              const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*,
                              const float*, const float*, const uint8_t*, float*, const bf16_t*,
                              const float*, const float*, float*, hipStream_t);
void dtf_gemm_stream_probe(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, hipStream_t);
void dtf_gemm_stream_pre(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, const float*,
                         const float*, bf16_t*, float*, hipStream_t, int);
void dtf_gemm_set_stagger(int, int);
void dtf_gemm_set_group(int);
int dtf_wgrad_get_pipe();
void dtf_lds_probe(int, int, int*, int, hipStream_t);
int dtf_max_dynamic_lds(int);
// transformer kernels (nlp.hip)
void dtf_ln_fwd(const bf16_t*, const float*, const bf16_t*, const float*, const float*, bf16_t*,
                bf16_t*, float*, float*, int, int, float, float, uint32_t, float, uint32_t,
                const int64_t*, const int64_t*, const bf16_t*, const bf16_t*, const bf16_t*, int,
                hipStream_t);
int dtf_ln_bwd_blocks(int);
void dtf_ln_set_wide(int);
void dtf_ln_bwd(const bf16_t*, const bf16_t*, const float*, const float*, const float*, bf16_t*,
                bf16_t*, float*, float*, float*, float*, int, int, float, uint32_t, float,
                uint32_t, hipStream_t, int);
void dtf_bias_gelu_fwd(const bf16_t*, const float*, bf16_t*, long, int, hipStream_t);
int dtf_bias_gelu_bwd_blocks(int);
int dtf_bf16_col_sum_ws_floats(int);
void dtf_bf16_col_sum(const bf16_t*, int, int, float*, float*, int, hipStream_t);
void dtf_slab_reduce(const float*, float*, long, int, int, hipStream_t);
// fused first-stage c3 backward (conv1x1_bwd.hip)
bool dtf_conv1x1_bwd_ok(int, int, int);
int dtf_conv1x1_bwd_blocks(int, int);
void dtf_conv1x1_bwd_set_grid(int);
void dtf_conv1x1_bwd_set_w16(int);
bool dtf_conv1x1_bwd_lazy_ok(int, int, int);
int dtf_conv1x1_bwd_lazy_blocks(int, int);
void dtf_conv1x1_bwd_lazy(const bf16_t*, const bf16_t*, const uint8_t*, const float*, const float*,
                          const float*, const bf16_t*, const bf16_t*, const bf16_t*, const float*,
                          const float*, const float*, const float*, bf16_t*, float*, float*, int,
                          int, int, const bf16_t*, hipStream_t);
void dtf_conv1x1_bwd(const bf16_t*, const bf16_t*, const bf16_t*, const bf16_t*, const float*,
                     const float*, const float*, const float*, bf16_t*, float*, float*, int, int,
                     int, hipStream_t);
void dtf_bias_gelu_bwd(const bf16_t*, const bf16_t*, const float*, bf16_t*, float*, float*, int,
                       int, hipStream_t, int);
void dtf_attn_fwd(const bf16_t*, const float*, bf16_t*, float*, int, int, int, float, float,
                  uint32_t, hipStream_t, uint32_t*);
long dtf_attn_keep_words(int, int, int, float);
void dtf_attn_set_keep(int);
void dtf_attn_bwd(const bf16_t*, const float*, const bf16_t*, const bf16_t*, const float*, float*,
                  bf16_t*, int, int, int, float, float, uint32_t, hipStream_t, float*,
                  const uint32_t*);
int dtf_attn_bwd_fused(int);
int dtf_pos_type_grad_ws_floats(int, int, int);
void dtf_attn_set_wide(int);
void dtf_attn_set_fused(int);
void dtf_pos_type_grad(const bf16_t*, const int64_t*, int, int, int, int, float*, float*, float*,
                       hipStream_t);
void dtf_segment_sum(const int64_t*, const int64_t*, const bf16_t*, float*, int, int,
                     hipStream_t);
void dtf_mlm_xent(const bf16_t*, const int64_t*, const float*, const float*, int, int, int,
                  float*, bf16_t*, hipStream_t);

// ---- dense GEMM (gemm.hip)
void dtf_gemm_nt_bias_gelu(const bf16_t*, const bf16_t*, bf16_t*, bf16_t*, int, int, int, int,
                           int, const float*, hipStream_t);
void dtf_gemm_nt_gelu_bwd(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int,
                          const bf16_t*, const float*, float*, hipStream_t);
void dtf_gemm_nt(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int,
                 const float*, const bf16_t*, int, float*, hipStream_t, const bf16_t*,
                 const uint8_t*);
int dtf_gemm_tile_rows(int);
void dtf_gemm_set_variant(int);
void dtf_gemm_set_pp(int);
void dtf_gemm_set_pp2(int);
int dtf_gemm_get_pp2();
bool dtf_gemm_pp2_ok(int M, int N, int K, int lda, int ldb);
int dtf_bias_relu_bwd_ws_floats(int);
void dtf_gather_u8_scale(const uint8_t*, const int64_t*, void*, int, int, float, int, hipStream_t);
// ---- fp32 path (f32.hip)
void dtf_gemm_f32(const float*, const float*, float*, const float*, int, int, int, long, long,
                  long, long, long, long, float, int, int, float*, hipStream_t);
int dtf_gemm_f32_splits(int, int, int);
void dtf_im2col_f32(const float*, float*, int, int, int, int, int, int, int, int, int, int, int,
                    int, hipStream_t);
void dtf_col2im_f32(const float*, float*, int, int, int, int, int, int, int, int, int, int, int,
                    int, hipStream_t);
void dtf_maxpool_f32_fwd(const float*, float*, uint8_t*, int, int, int, int, int, int, int, int,
                         hipStream_t);
void dtf_maxpool_f32_bwd(const float*, const uint8_t*, float*, int, int, int, int, int, int, int,
                         int, hipStream_t);
int dtf_bias_relu_bwd_f32_ws_floats(int);
void dtf_bias_relu_bwd_f32(const float*, const float*, float*, int, int, float*, float*, int, int,
                           hipStream_t);
void dtf_clipped_xent(const float*, const float*, int, int, float*, float*, float, hipStream_t);
void dtf_bias_relu_bwd(const bf16_t*, const bf16_t*, bf16_t*, int, int, float*, float*, int, int,
                       hipStream_t);

// ---- HIP IPC buffers (ipc.cpp) handed to torch as DLPack capsules
uintptr_t dtf_ipc_alloc(size_t, int);
std::string dtf_ipc_handle(uintptr_t, int);
uintptr_t dtf_ipc_open(const std::string&, int);
void dtf_ipc_close(uintptr_t, int);
void dtf_ipc_free(uintptr_t, int);

namespace dlp {   // DLPack ABI (v0.8 DLManagedTensor, "dltensor" capsule)
struct Device { int32_t device_type; int32_t device_id; };
struct DataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct Tensor { void* data; Device device; int32_t ndim; DataType dtype; int64_t* shape;
                int64_t* strides; uint64_t byte_offset; };
struct Managed { Tensor t; void* ctx; void (*deleter)(Managed*); };
constexpr int32_t kROCM = 10;
struct Ctx { int64_t shape[1]; int64_t strides[1]; uintptr_t ptr; int device; bool opened; };
void deleter(Managed* m) {
  auto* c = static_cast<Ctx*>(m->ctx);
  if (c->opened) dtf_ipc_close(c->ptr, c->device);
  else dtf_ipc_free(c->ptr, c->device);
  delete c;
  delete m;
}
void capsule_destructor(PyObject* cap) {   // capsule dropped without being consumed by torch
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* m = static_cast<Managed*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (m && m->deleter) m->deleter(m);
  }
}
// 1-D float32 (or uint8 when dtype_bits == 8) view of an IPC buffer as a DLPack capsule
py::capsule make(uintptr_t ptr, int64_t numel, int device, bool opened, int dtype_bits) {
  auto* c = new Ctx{{numel}, {1}, ptr, device, opened};
  auto* m = new Managed{};
  m->t.data = reinterpret_cast<void*>(ptr);
  m->t.device = {kROCM, device};
  m->t.ndim = 1;
  m->t.dtype = dtype_bits == 8 ? DataType{1, 8, 1} : DataType{2, 32, 1};
  m->t.shape = c->shape;
  m->t.strides = c->strides;
  m->t.byte_offset = 0;
  m->ctx = c;
  m->deleter = deleter;
  return py::reinterpret_steal<py::capsule>(PyCapsule_New(m, "dltensor", capsule_destructor));
}
}  // namespace dlp

template <typename T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename TT>
static TT make_taps(const std::vector<int>& dh, const std::vector<int>& dw) {
  if (dh.size() != dw.size() || dh.empty() || dh.size() > DTF_MAX_TAPS)
    throw std::runtime_error("bad tap table");
  TT t{};
  t.n = (int)dh.size();
  for (size_t i = 0; i < dh.size(); ++i) { t.dh[i] = dh[i]; t.dw[i] = dw[i]; }
  return t;
}

// rccl_comm.cpp: native RCCL communicator
int dtf_rccl_load(const std::string& path);
std::string dtf_rccl_unique_id();
long dtf_rccl_comm_init(const std::string& uid, int nranks, int rank, int device);
void dtf_rccl_comm_destroy(long comm, int abort);
int dtf_rccl_async_error(long comm);
void dtf_rccl_all_reduce(long comm, long send, long recv, long count, int dtype, int op, long stream);
void dtf_rccl_reduce_scatter(long comm, long send, long recv, long recvcount, int dtype, int op,
                             long stream);
void dtf_rccl_all_gather(long comm, long send, long recv, long sendcount, int dtype, long stream);
void dtf_rccl_broadcast(long comm, long send, long recv, long count, int dtype, int root, long stream);
void dtf_rccl_reduce(long comm, long send, long recv, long count, int dtype, int op, int root,
                     long stream);
void dtf_rccl_group(int start);

PYBIND11_MODULE(_dtf_hip, m) {
  m.def("rccl_load", &dtf_rccl_load);
  m.def("rccl_unique_id", []() { return py::bytes(dtf_rccl_unique_id()); });
  m.def("rccl_comm_init", &dtf_rccl_comm_init);
  m.def("rccl_comm_destroy", &dtf_rccl_comm_destroy);
  m.def("rccl_async_error", &dtf_rccl_async_error);
  m.def("rccl_all_reduce", &dtf_rccl_all_reduce);
  m.def("rccl_reduce_scatter", &dtf_rccl_reduce_scatter);
  m.def("rccl_all_gather", &dtf_rccl_all_gather);
  m.def("rccl_broadcast", &dtf_rccl_broadcast);
  m.def("rccl_reduce", &dtf_rccl_reduce);
  m.def("rccl_group", &dtf_rccl_group);
  m.doc() = "distributedtensorflow_amd HIP/CDNA4 kernels (gfx950)";

  m.def("gemm_nt", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K, int lda,
                      int ldb, int ldc, uintptr_t bias, uintptr_t cin, int relu, uintptr_t st,
                      uintptr_t stats, uintptr_t acc_src, uintptr_t acc_mask) {
    dtf_gemm_nt(P<bf16_t>(a), P<bf16_t>(b), P<bf16_t>(c), M, N, K, lda, ldb, ldc,
                P<float>(bias), P<bf16_t>(cin), relu, P<float>(stats), S(st), P<bf16_t>(acc_src),
                P<uint8_t>(acc_mask));
    check_launch("gemm_nt");
  }, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("M"), py::arg("N"), py::arg("K"),
     py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("bias"), py::arg("cin"),
     py::arg("relu"), py::arg("stream"), py::arg("stats") = 0, py::arg("acc_src") = 0,
     py::arg("acc_mask") = 0);
  m.def("gemm_nt_bias_gelu", [](uintptr_t a, uintptr_t b, uintptr_t z, uintptr_t h, int M, int N,
                                int K, int lda, int ldb, uintptr_t bias, uintptr_t st) {
    dtf_gemm_nt_bias_gelu(P<bf16_t>(a), P<bf16_t>(b), P<bf16_t>(z), P<bf16_t>(h), M, N, K, lda,
                          ldb, P<float>(bias), S(st));
    check_launch("gemm_nt_bias_gelu");
  });
  m.def("gemm_nt_gelu_bwd", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K,
                               int lda, int ldb, uintptr_t gelu_a, uintptr_t gelu_b,
                               uintptr_t colsum, uintptr_t st) {
    dtf_gemm_nt_gelu_bwd(P<bf16_t>(a), P<bf16_t>(b), P<bf16_t>(c), M, N, K, lda, ldb,
                         P<bf16_t>(gelu_a), P<float>(gelu_b), P<float>(colsum), S(st));
    check_launch("gemm_nt_gelu_bwd");
  });
  m.def("gemm_tile_rows", &dtf_gemm_tile_rows);
  m.def("gemm_set_variant", &dtf_gemm_set_variant);
  m.def("gemm_set_pp", &dtf_gemm_set_pp);
  m.def("gemm_set_pp2", &dtf_gemm_set_pp2);
  m.def("gemm_get_pp2", &dtf_gemm_get_pp2);
  m.def("gemm_pp2_ok", &dtf_gemm_pp2_ok);
  m.def("bias_relu_bwd_ws_floats", &dtf_bias_relu_bwd_ws_floats);
  m.def("gather_u8_scale", [](uintptr_t images, uintptr_t idx, uintptr_t out, int B, int D,
                              float scale, int out_bf16, uintptr_t st) {
    dtf_gather_u8_scale(P<uint8_t>(images), P<int64_t>(idx), P<void>(out), B, D, scale, out_bf16,
                        S(st));
    check_launch("gather_u8_scale");
  });
  m.def("gemm_f32_splits", &dtf_gemm_f32_splits);
  m.def("gemm_f32", [](uintptr_t a, uintptr_t b, uintptr_t c, uintptr_t bias, int M, int N, int K,
                       long sam, long sak, long sbn, long sbk, long scm, long scn, float alpha,
                       int relu, int accumulate, uintptr_t ws, uintptr_t st) {
    dtf_gemm_f32(P<float>(a), P<float>(b), P<float>(c), P<float>(bias), M, N, K, sam, sak, sbn,
                 sbk, scm, scn, alpha, relu, accumulate, P<float>(ws), S(st));
    check_launch("gemm_f32");
  });
  m.def("im2col_f32", [](uintptr_t x, uintptr_t cols, int N, int H, int W, int C, int P_, int Q,
                         int sh, int sw, int R, int S_, int pt, int pl, uintptr_t st) {
    dtf_im2col_f32(P<float>(x), P<float>(cols), N, H, W, C, P_, Q, sh, sw, R, S_, pt, pl, S(st));
    check_launch("im2col_f32");
  });
  m.def("col2im_f32", [](uintptr_t dc, uintptr_t dx, int N, int H, int W, int C, int P_, int Q,
                         int sh, int sw, int R, int S_, int pt, int pl, uintptr_t st) {
    dtf_col2im_f32(P<float>(dc), P<float>(dx), N, H, W, C, P_, Q, sh, sw, R, S_, pt, pl, S(st));
    check_launch("col2im_f32");
  });
  m.def("maxpool_f32_fwd", [](uintptr_t x, uintptr_t y, uintptr_t arg, int N, int H, int W, int C,
                              int P_, int Q, int k, int s, uintptr_t st) {
    dtf_maxpool_f32_fwd(P<float>(x), P<float>(y), P<uint8_t>(arg), N, H, W, C, P_, Q, k, s, S(st));
    check_launch("maxpool_f32_fwd");
  });
  m.def("maxpool_f32_bwd", [](uintptr_t dy, uintptr_t arg, uintptr_t dx, int N, int H, int W,
                              int C, int P_, int Q, int k, int s, uintptr_t st) {
    dtf_maxpool_f32_bwd(P<float>(dy), P<uint8_t>(arg), P<float>(dx), N, H, W, C, P_, Q, k, s, S(st));
    check_launch("maxpool_f32_bwd");
  });
  m.def("bias_relu_bwd_f32_ws_floats", &dtf_bias_relu_bwd_f32_ws_floats);
  m.def("bias_relu_bwd_f32", [](uintptr_t dy, uintptr_t y, uintptr_t dz, int T, int N,
                                uintptr_t ws, uintptr_t db, int accumulate, int relu, uintptr_t st) {
    dtf_bias_relu_bwd_f32(P<float>(dy), P<float>(y), P<float>(dz), T, N, P<float>(ws),
                          P<float>(db), accumulate, relu, S(st));
    check_launch("bias_relu_bwd_f32");
  });
  m.def("clipped_xent", [](uintptr_t z, uintptr_t t, int B, int V, uintptr_t rows, uintptr_t dz,
                           float scale, uintptr_t st) {
    dtf_clipped_xent(P<float>(z), P<float>(t), B, V, P<float>(rows), P<float>(dz), scale, S(st));
    check_launch("clipped_xent");
  });
  m.def("bias_relu_bwd", [](uintptr_t dy, uintptr_t y, uintptr_t dz, int T, int N, uintptr_t ws,
                            uintptr_t db, int accumulate, int relu, uintptr_t st) {
    dtf_bias_relu_bwd(P<bf16_t>(dy), P<bf16_t>(y), P<bf16_t>(dz), T, N, P<float>(ws), P<float>(db),
                      accumulate, relu, S(st));
    check_launch("bias_relu_bwd");
  });
  // parameter-server data plane: exported / mapped HBM buffers (ipc.cpp)
  m.def("ipc_alloc", [](int64_t numel, int device, int dtype_bits) {
    const size_t bytes = (size_t)numel * (dtype_bits == 8 ? 1 : 4);
    uintptr_t p = dtf_ipc_alloc(bytes, device);
    py::bytes h(dtf_ipc_handle(p, device));
    return py::make_tuple(dlp::make(p, numel, device, false, dtype_bits), h);
  }, py::arg("numel"), py::arg("device"), py::arg("dtype_bits") = 32);
  m.def("ipc_open", [](py::bytes handle, int64_t numel, int device, int dtype_bits) {
    uintptr_t p = dtf_ipc_open(std::string(handle), device);
    return dlp::make(p, numel, device, true, dtype_bits);
  }, py::arg("handle"), py::arg("numel"), py::arg("device"), py::arg("dtype_bits") = 32);

  m.def("bn_partial_blocks", &dtf_bn_partial_blocks);
  m.def("bn_workspace_floats", &dtf_bn_workspace_floats);
  m.def("bn_workspace_floats_g", &dtf_bn_workspace_floats_g);
  m.def("conv_stats_rows", &dtf_conv_stats_rows, py::arg("M"), py::arg("Kout"), py::arg("C") = 0,
        py::arg("taps") = 1, py::arg("W") = 0);
  m.def("conv_set_halo", &dtf_conv_set_halo);
  // a probe build (-DDTF_PROBES) carries wrong-result timing probes: bench.py / smoke() refuse it
  m.def("probes_built", []() {
#ifdef DTF_PROBES
    return true;
#else
    return false;
#endif
  });
  m.def("conv_set_bnl_probe", &dtf_conv_set_bnl_probe);
  m.def("gemm_stream_set_bnb_probe", &dtf_gemm_stream_set_bnb_probe);
  m.def("conv_tile_rows", [](std::vector<int> geom, std::vector<int> dh, std::vector<int> dw,
                             int bnb) {
    if (geom.size() != 16 && geom.size() != 17)
      throw std::runtime_error("conv_tile_rows: geom needs 16 (+acc) ints");
    ConvGeom g{geom[0], geom[1], geom[2],  geom[3],  geom[4],  geom[5],  geom[6],  geom[7],
               geom[8], geom[9], geom[10], geom[11], geom[12], geom[13], geom[14], geom[15],
               geom.size() == 17 ? geom[16] : 0};
    return dtf_conv_tile_rows(g, make_taps<TapTable>(dh, dw), bnb);
  }, py::arg("geom"), py::arg("dh"), py::arg("dw"), py::arg("bnb") = 0);
  m.def("conv_set_halo_bnb", &dtf_conv_set_halo_bnb);
  m.def("conv_set_dma_mode", &dtf_conv_set_dma_mode);
  m.def("filter_transpose", [](std::vector<uintptr_t> src, std::vector<uintptr_t> dst,
                               std::vector<int> K, std::vector<int> T, std::vector<int> C,
                               uintptr_t st) {
    // [K][T][C] -> [C][T][K] for every job, kWtMaxJobs per launch
    const size_t n = src.size();
    if (dst.size() != n || K.size() != n || T.size() != n || C.size() != n)
      throw std::runtime_error("filter_transpose: ragged job lists");
    for (size_t b = 0; b < n; b += kWtMaxJobs) {
      WtJobs j{};
      int tiles = 0;
      j.n = (int)std::min(n - b, (size_t)kWtMaxJobs);
      for (int i = 0; i < j.n; ++i) {
        const size_t q = b + i;
        if (K[q] <= 0 || T[q] <= 0 || C[q] <= 0) throw std::runtime_error("filter_transpose: bad dims");
        j.src[i] = P<const bf16_t>(src[q]);
        j.dst[i] = P<bf16_t>(dst[q]);
        j.K[i] = K[q]; j.T[i] = T[q]; j.C[i] = C[q];
        tiles += T[q] * ((K[q] + 63) / 64) * ((C[q] + 63) / 64);
        j.tile_end[i] = tiles;
      }
      dtf_filter_transpose(j, S(st));
      check_launch("filter_transpose");
    }
  });
  m.def("conv_set_stem_halo", &dtf_conv_set_stem_halo);
  m.def("conv_set_halo_strips", &dtf_conv_set_halo_strips);
  m.def("conv_set_halo_freg", &dtf_conv_set_halo_freg);
  m.def("conv_set_small_k", &dtf_conv_set_small_k);
  m.def("bn_fwd_finalize_g", [](uintptr_t part, int G, long M, int C, uintptr_t gamma,
                                uintptr_t beta, uintptr_t rm, uintptr_t rv, float mom, float eps,
                                uintptr_t mean, uintptr_t invstd, uintptr_t scale, uintptr_t shift,
                                uintptr_t st) {
    dtf_bn_fwd_finalize_g(P<const float>(part), G, M, C, P<const float>(gamma),
                          P<const float>(beta), P<float>(rm), P<float>(rv), mom, eps,
                          P<float>(mean), P<float>(invstd), P<float>(scale), P<float>(shift),
                          S(st));
    check_launch("bn_fwd_finalize_g");
  });
  m.def("bn_fwd_stats", [](uintptr_t x, long M, int C, uintptr_t part, uintptr_t st) {
    dtf_bn_fwd_stats(P<const bf16_t>(x), M, C, P<float>(part), S(st));
    check_launch("bn_fwd_stats");
  });
  m.def("bn_fwd_finalize", [](uintptr_t part, long M, int C, uintptr_t gamma, uintptr_t beta,
                              uintptr_t rm, uintptr_t rv, float mom, float eps, uintptr_t mean,
                              uintptr_t invstd, uintptr_t scale, uintptr_t shift, uintptr_t st) {
    dtf_bn_fwd_finalize(P<const float>(part), M, C, P<const float>(gamma), P<const float>(beta),
                        P<float>(rm), P<float>(rv), mom, eps, P<float>(mean), P<float>(invstd),
                        P<float>(scale), P<float>(shift), S(st));
    check_launch("bn_fwd_finalize");
  });
  m.def("bn_infer_finalize", [](int C, uintptr_t gamma, uintptr_t beta, uintptr_t rm,
                                uintptr_t rv, float eps, uintptr_t mean, uintptr_t invstd,
                                uintptr_t scale, uintptr_t shift, uintptr_t st) {
    dtf_bn_infer_finalize(C, P<const float>(gamma), P<const float>(beta), P<const float>(rm),
                          P<const float>(rv), eps, P<float>(mean), P<float>(invstd),
                          P<float>(scale), P<float>(shift), S(st));
    check_launch("bn_infer_finalize");
  });
  m.def("bn_apply", [](uintptr_t x, uintptr_t res, uintptr_t y, uintptr_t scale, uintptr_t shift,
                       long M, int C, int relu, uintptr_t st, uintptr_t mask) {
    dtf_bn_apply(P<const bf16_t>(x), P<const bf16_t>(res), P<bf16_t>(y), P<uint8_t>(mask),
                 P<const float>(scale), P<const float>(shift), M, C, relu, S(st));
    check_launch("bn_apply");
  }, py::arg("x"), py::arg("res"), py::arg("y"), py::arg("scale"), py::arg("shift"), py::arg("M"),
     py::arg("C"), py::arg("relu"), py::arg("stream"), py::arg("mask") = 0);
  m.def("bn_bwd_reduce", [](uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t mean,
                            uintptr_t invstd, long M, int C, int relu, uintptr_t part,
                            uintptr_t st, uintptr_t fsc, uintptr_t fsh, uintptr_t mask) {
    dtf_bn_bwd_reduce(P<const bf16_t>(dy), P<const bf16_t>(y), P<const uint8_t>(mask),
                      P<const bf16_t>(x), P<const float>(mean), P<const float>(invstd), M, C, relu,
                      P<float>(part), P<const float>(fsc), P<const float>(fsh), S(st));
    check_launch("bn_bwd_reduce");
  }, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("mean"), py::arg("invstd"), py::arg("M"),
     py::arg("C"), py::arg("relu"), py::arg("part"), py::arg("stream"), py::arg("scale") = 0,
     py::arg("shift") = 0, py::arg("mask") = 0);
  m.def("bn_bwd_finalize", [](uintptr_t part, long M, int C, uintptr_t gamma, uintptr_t mean,
                              uintptr_t invstd, uintptr_t dg, uintptr_t db, uintptr_t a,
                              uintptr_t b, uintptr_t c, int accumulate, uintptr_t st) {
    dtf_bn_bwd_finalize(P<const float>(part), M, C, P<const float>(gamma), P<const float>(mean),
                        P<const float>(invstd), P<float>(dg), P<float>(db), P<float>(a),
                        P<float>(b), P<float>(c), accumulate, S(st));
    check_launch("bn_bwd_finalize");
  });
  m.def("bn_apply_dual", [](uintptr_t x, uintptr_t xp, uintptr_t y, uintptr_t mask,
                            uintptr_t scale, uintptr_t shift, uintptr_t pscale, uintptr_t pshift,
                            long M, int C, int relu, uintptr_t st) {
    dtf_bn_apply_dual(P<const bf16_t>(x), P<const bf16_t>(xp), P<bf16_t>(y), P<uint8_t>(mask),
                      P<const float>(scale), P<const float>(shift), P<const float>(pscale),
                      P<const float>(pshift), M, C, relu, S(st));
    check_launch("bn_apply_dual");
  });
  m.def("bn_bwd_reduce_dual", [](uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t mean,
                                 uintptr_t invstd, uintptr_t xp, uintptr_t meanp,
                                 uintptr_t invstdp, long M, int C, uintptr_t part,
                                 uintptr_t partp, uintptr_t st) {
    dtf_bn_bwd_reduce_dual(P<const bf16_t>(dy), P<const uint8_t>(mask), P<const bf16_t>(x),
                           P<const float>(mean), P<const float>(invstd), P<const bf16_t>(xp),
                           P<const float>(meanp), P<const float>(invstdp), M, C, P<float>(part),
                           P<float>(partp), S(st));
    check_launch("bn_bwd_reduce_dual");
  });
  m.def("bn_bwd_apply_dual", [](uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t a,
                                uintptr_t b, uintptr_t c, uintptr_t dx, uintptr_t xp,
                                uintptr_t ap, uintptr_t bp, uintptr_t cp, uintptr_t dxp, long M,
                                int C, uintptr_t st) {
    dtf_bn_bwd_apply_dual(P<const bf16_t>(dy), P<const uint8_t>(mask), P<const bf16_t>(x),
                          P<const float>(a), P<const float>(b), P<const float>(c), P<bf16_t>(dx),
                          P<const bf16_t>(xp), P<const float>(ap), P<const float>(bp),
                          P<const float>(cp), P<bf16_t>(dxp), M, C, S(st));
    check_launch("bn_bwd_apply_dual");
  });
  m.def("relu_mask_apply", [](uintptr_t dy, uintptr_t mask, uintptr_t out, long n, uintptr_t st) {
    dtf_relu_mask_apply(P<const bf16_t>(dy), P<const uint8_t>(mask), P<bf16_t>(out), n, S(st));
    check_launch("relu_mask_apply");
  });
  m.def("bn_bwd_apply", [](uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t a, uintptr_t b,
                           uintptr_t c, uintptr_t dx, uintptr_t dres, long M, int C, int relu,
                           uintptr_t st, uintptr_t fsc, uintptr_t fsh, uintptr_t mask) {
    dtf_bn_bwd_apply(P<const bf16_t>(dy), P<const bf16_t>(y), P<const uint8_t>(mask),
                     P<const bf16_t>(x), P<const float>(a), P<const float>(b), P<const float>(c),
                     P<bf16_t>(dx), P<bf16_t>(dres), M, C, relu, P<const float>(fsc),
                     P<const float>(fsh), S(st));
    check_launch("bn_bwd_apply");
  }, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("a"), py::arg("b"), py::arg("c"),
     py::arg("dx"), py::arg("dres"), py::arg("M"), py::arg("C"), py::arg("relu"),
     py::arg("stream"), py::arg("scale") = 0, py::arg("shift") = 0, py::arg("mask") = 0);
  m.def("maxpool_fwd", [](uintptr_t x, uintptr_t y, uintptr_t arg, int N, int H, int W, int C,
                          int Pp, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                          uintptr_t st) {
    dtf_maxpool_fwd(P<const bf16_t>(x), P<bf16_t>(y), P<uint8_t>(arg), N, H, W, C, Pp, Q, kh, kw,
                    sh, sw, ph, pw, S(st));
    check_launch("maxpool_fwd");
  });
  m.def("maxpool_bwd", [](uintptr_t dy, uintptr_t arg, uintptr_t dx, int N, int H, int W, int C,
                          int Pp, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                          uintptr_t st) {
    dtf_maxpool_bwd(P<const bf16_t>(dy), P<const uint8_t>(arg), P<bf16_t>(dx), N, H, W, C, Pp, Q,
                    kh, kw, sh, sw, ph, pw, S(st));
    check_launch("maxpool_bwd");
  });
  m.def("gap_fwd", [](uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t st) {
    dtf_gap_fwd(P<const bf16_t>(x), P<bf16_t>(y), N, HW, C, S(st));
    check_launch("gap_fwd");
  });
  m.def("bn_relu_maxpool_fwd", [](uintptr_t x, uintptr_t scale, uintptr_t shift, uintptr_t y,
                                  uintptr_t arg, int N, int H, int W, int C, int P_, int Q,
                                  int kh, int kw, int sh, int sw, int ph, int pw, uintptr_t st) {
    dtf_bn_relu_maxpool_fwd(P<const bf16_t>(x), P<const float>(scale), P<const float>(shift),
                            P<bf16_t>(y), P<uint8_t>(arg), N, H, W, C, P_, Q, kh, kw, sh, sw, ph,
                            pw, S(st));
    check_launch("bn_relu_maxpool_fwd");
  });
  m.def("pool_set_blocked", &dtf_pool_set_blocked);
  m.def("s2d_set_rows", &dtf_s2d_set_rows);
  m.def("pool_bn_bwd_blocks", &dtf_pool_bn_bwd_blocks);
  m.def("pool_bn_bwd_set_caps", &dtf_pool_bn_bwd_set_caps);
  m.def("pool_bn_bwd_reduce", [](uintptr_t dy, uintptr_t arg, uintptr_t x, uintptr_t mean,
                                 uintptr_t invstd, uintptr_t fsc, uintptr_t fsh, uintptr_t part,
                                 int N, int H, int W, int C, int P_, int Q, uintptr_t st) {
    dtf_pool_bn_bwd_reduce(P<const bf16_t>(dy), P<const uint8_t>(arg), P<const bf16_t>(x),
                           P<const float>(mean), P<const float>(invstd), P<const float>(fsc),
                           P<const float>(fsh), P<float>(part), N, H, W, C, P_, Q, S(st));
    check_launch("pool_bn_bwd_reduce");
  });
  m.def("pool_bn_bwd_apply", [](uintptr_t dy, uintptr_t arg, uintptr_t x, uintptr_t a,
                                uintptr_t b, uintptr_t c, uintptr_t fsc, uintptr_t fsh,
                                uintptr_t dx, int N, int H, int W, int C, int P_, int Q,
                                uintptr_t st) {
    dtf_pool_bn_bwd_apply(P<const bf16_t>(dy), P<const uint8_t>(arg), P<const bf16_t>(x),
                          P<const float>(a), P<const float>(b), P<const float>(c),
                          P<const float>(fsc), P<const float>(fsh), P<bf16_t>(dx), N, H, W, C,
                          P_, Q, S(st));
    check_launch("pool_bn_bwd_apply");
  });
  m.def("s2d_input", [](uintptr_t x, uintptr_t xs, int N, int H, int W, int C, int Ho, int Wo,
                        int s_, int cp, int pad, uintptr_t st) {
    dtf_s2d_input(P<const bf16_t>(x), P<bf16_t>(xs), N, H, W, C, Ho, Wo, s_, cp, pad, S(st));
    check_launch("s2d_input");
  });
  m.def("gap_bwd", [](uintptr_t dy, uintptr_t dx, int N, int HW, int C, uintptr_t st) {
    dtf_gap_bwd(P<const bf16_t>(dy), P<bf16_t>(dx), N, HW, C, S(st));
    check_launch("gap_bwd");
  });
  m.def("softmax_xent", [](uintptr_t logits, uintptr_t labels, int label_bytes, int B, int V,
                           uintptr_t loss_rows, uintptr_t grad, float gscale, uintptr_t st) {
    dtf_softmax_xent(P<const float>(logits), P<const void>(labels), label_bytes, B, V,
                     P<float>(loss_rows), P<float>(grad), gscale, S(st));
    check_launch("softmax_xent");
  });
  m.def("sgd_momentum", [](uintptr_t p, uintptr_t g, uintptr_t a, uintptr_t shadow, long n,
                           uintptr_t lr, float mom, float wd, float gscale, int nesterov,
                           uintptr_t nonfinite, uintptr_t st) {
    dtf_sgd_momentum(P<float>(p), P<const float>(g), P<float>(a), P<bf16_t>(shadow), n,
                     P<const float>(lr), mom, wd, gscale, nesterov, P<int>(nonfinite), S(st));
    check_launch("sgd_momentum");
  });
  m.def("adam", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t shadow, long n,
                   uintptr_t lr_t, float b1, float b2, float eps, float wd, float gscale,
                   uintptr_t nonfinite, uintptr_t st) {
    dtf_adam(P<float>(p), P<const float>(g), P<float>(mm), P<float>(v), P<bf16_t>(shadow), n,
             P<const float>(lr_t), b1, b2, eps, wd, gscale, P<int>(nonfinite), S(st));
    check_launch("adam");
  });
  m.def("adagrad", [](uintptr_t p, uintptr_t g, uintptr_t acc, uintptr_t shadow, long n,
                      uintptr_t lr, float gscale, uintptr_t nonfinite, uintptr_t st) {
    dtf_adagrad(P<float>(p), P<const float>(g), P<float>(acc), P<bf16_t>(shadow), n,
                P<const float>(lr), gscale, P<int>(nonfinite), S(st));
    check_launch("adagrad");
  });
  m.def("lamb", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t shadow,
                   uintptr_t chunks, int nchunks, uintptr_t hyper, uintptr_t lr, float b1,
                   float b2, float eps, uintptr_t wd_seg, float gscale, uintptr_t norms,
                   uintptr_t nonfinite, uintptr_t st) {
    dtf_lamb(P<float>(p), P<float>(g), P<float>(mm), P<float>(v), P<bf16_t>(shadow),
             P<const void>(chunks), nchunks, P<const float>(hyper), P<const float>(lr), b1, b2,
             eps, P<const float>(wd_seg), gscale, P<float>(norms), P<int>(nonfinite), S(st));
    check_launch("lamb");
  });
  m.def("lamb_chunk_bytes", &dtf_lamb_chunk_bytes);
  m.def("sumsq", [](uintptr_t x, long n, uintptr_t out, uintptr_t st) {
    dtf_sumsq(P<const float>(x), n, P<float>(out), S(st));
    check_launch("sumsq");
  });
  m.def("cast_f32_bf16", [](uintptr_t x, uintptr_t y, long n, uintptr_t st) {
    dtf_cast_f32_bf16(P<const float>(x), P<bf16_t>(y), n, S(st));
    check_launch("cast_f32_bf16");
  });
  m.def("conv_igemm", [](uintptr_t x, uintptr_t w, uintptr_t y, std::vector<int> geom,
                         std::vector<int> dh, std::vector<int> dw, int bk, uintptr_t st,
                         uintptr_t stats, std::vector<uintptr_t> bnb, uintptr_t acc_src,
                         uintptr_t acc_mask, uintptr_t bias, int relu, uintptr_t bnl_sc,
                         uintptr_t bnl_sh, uintptr_t bnl_y) {
    if (geom.size() != 16 && geom.size() != 17)
      throw std::runtime_error("conv_igemm: geom needs 16 (+acc) ints");
    ConvGeom g{geom[0], geom[1], geom[2],  geom[3],  geom[4],  geom[5],  geom[6],  geom[7],
               geom[8], geom[9], geom[10], geom[11], geom[12], geom[13], geom[14], geom[15],
               geom.size() == 17 ? geom[16] : 0, P<const bf16_t>(acc_src),
               P<const uint8_t>(acc_mask), P<const float>(bias), relu};
    if (g.acc == 2 && (!g.acc_src || !g.acc_mask))
      throw std::runtime_error("conv_igemm: acc 2 needs acc_src and acc_mask");
    g.lsc = P<const float>(bnl_sc);
    g.lsh = P<const float>(bnl_sh);
    g.ly = P<bf16_t>(bnl_y);
    // bnb = [x, mean, invstd, fsc, fsh, mask, part, mkind, row0] (fused BN-backward sums) or []
    BnBwdEpi e{};
    if (!bnb.empty()) {
      if (bnb.size() != 9) throw std::runtime_error("conv_igemm: bnb needs 9 entries");
      e = BnBwdEpi{P<const bf16_t>(bnb[0]), P<const float>(bnb[1]), P<const float>(bnb[2]),
                   P<const float>(bnb[3]), P<const float>(bnb[4]), P<const uint8_t>(bnb[5]),
                   P<float>(bnb[6]), (int)bnb[7], (int)bnb[8]};
    }
    dtf_conv_igemm(P<const bf16_t>(x), P<const bf16_t>(w), P<bf16_t>(y), g,
                   make_taps<TapTable>(dh, dw), bk, P<float>(stats), e, S(st));
    check_launch("conv_igemm");
  }, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("geom"), py::arg("dh"), py::arg("dw"),
     py::arg("bk"), py::arg("stream"), py::arg("stats") = 0,
     py::arg("bnb") = std::vector<uintptr_t>{}, py::arg("acc_src") = 0, py::arg("acc_mask") = 0,
     py::arg("bias") = 0, py::arg("relu") = 0, py::arg("bnl_sc") = 0, py::arg("bnl_sh") = 0,
     py::arg("bnl_y") = 0);
  // the phase classes of a strided data gradient in one launch; False: not eligible, nothing
  // launched (the caller launches the classes one by one)
  m.def("conv_igemm_grouped", [](uintptr_t x, uintptr_t y, std::vector<int> geom,
                                 std::vector<uintptr_t> wts, std::vector<int> oh0,
                                 std::vector<int> ow0, std::vector<int> kpad,
                                 std::vector<std::vector<int>> dh, std::vector<std::vector<int>> dw,
                                 uintptr_t st, std::vector<uintptr_t> bnb, std::vector<int> row0) {
    if (geom.size() != 17) throw std::runtime_error("conv_igemm_grouped: geom needs 17 ints");
    const size_t n = wts.size();
    if (oh0.size() != n || ow0.size() != n || kpad.size() != n || dh.size() != n ||
        dw.size() != n || (!bnb.empty() && row0.size() != n))
      throw std::runtime_error("conv_igemm_grouped: per-class lists differ in length");
    ConvGeom g{geom[0], geom[1], geom[2],  geom[3],  geom[4],  geom[5],  geom[6],  geom[7],
               geom[8], geom[9], geom[10], geom[11], geom[12], geom[13], geom[14], geom[15],
               geom[16]};
    BnBwdEpi e{};
    if (!bnb.empty()) {
      if (bnb.size() != 8) throw std::runtime_error("conv_igemm_grouped: bnb needs 8 entries");
      e = BnBwdEpi{P<const bf16_t>(bnb[0]), P<const float>(bnb[1]), P<const float>(bnb[2]),
                   P<const float>(bnb[3]), P<const float>(bnb[4]), P<const uint8_t>(bnb[5]),
                   P<float>(bnb[6]), (int)bnb[7], 0};
    }
    std::vector<const bf16_t*> w(n);
    for (size_t i = 0; i < n; ++i) w[i] = P<const bf16_t>(wts[i]);
    const bool ok = dtf_conv_igemm_grouped(P<const bf16_t>(x), P<bf16_t>(y), g, (int)n, w.data(),
                                           oh0.data(), ow0.data(), kpad.data(), dh, dw, e,
                                           row0.empty() ? nullptr : row0.data(), S(st));
    if (ok) check_launch("conv_igemm_grouped");
    return ok;
  });
  m.def("gemm_conv_part_images", &dtf_gemm_conv_part_images);
  m.def("gemm_set_pp2_strided", &dtf_gemm_set_pp2_strided);
  m.def("conv_bnl_ok", [](std::vector<int> geom, std::vector<int> dh, std::vector<int> dw) {
    if (geom.size() != 16 && geom.size() != 17)
      throw std::runtime_error("conv_bnl_ok: geom needs 16 (+acc) ints");
    ConvGeom g{geom[0], geom[1], geom[2],  geom[3],  geom[4],  geom[5],  geom[6],  geom[7],
               geom[8], geom[9], geom[10], geom[11], geom[12], geom[13], geom[14], geom[15],
               geom.size() == 17 ? geom[16] : 0};
    return dtf_conv_bnl_ok(g, make_taps<TapTable>(dh, dw));
  });
  m.def("bn_bwd_finalize_g", [](uintptr_t part, int G, long M, int C, uintptr_t gamma,
                                uintptr_t mean, uintptr_t invstd, uintptr_t dg, uintptr_t db,
                                uintptr_t a, uintptr_t b, uintptr_t c, int accumulate,
                                uintptr_t st) {
    dtf_bn_bwd_finalize_g(P<const float>(part), G, M, C, P<const float>(gamma),
                          P<const float>(mean), P<const float>(invstd), P<float>(dg), P<float>(db),
                          P<float>(a), P<float>(b), P<float>(c), accumulate, S(st));
    check_launch("bn_bwd_finalize_g");
  });
  m.def("conv_wgrad", [](uintptr_t x, uintptr_t dy, uintptr_t dw_out, uintptr_t ws,
                         std::vector<int> geom, std::vector<int> dh, std::vector<int> dw,
                         int splits, uintptr_t st, int tr_mode, int accumulate) {
    if (geom.size() != 10) throw std::runtime_error("conv_wgrad: geom needs 10 ints");
    WgradGeom g{geom[0], geom[1], geom[2], geom[3], geom[4], geom[5], geom[6], geom[7], geom[8],
                geom[9], 0, 0};
    dtf_conv_wgrad(P<const bf16_t>(x), P<const bf16_t>(dy), P<float>(dw_out), P<float>(ws), g,
                   make_taps<TapTableW>(dh, dw), splits, tr_mode, accumulate, S(st));
    check_launch("conv_wgrad");
  }, py::arg("x"), py::arg("dy"), py::arg("dw_out"), py::arg("ws"), py::arg("geom"),
     py::arg("dh"), py::arg("dw"), py::arg("splits"), py::arg("stream"), py::arg("tr_mode") = 1,
     py::arg("accumulate") = 0);
  m.def("conv_wgrad_splits", &dtf_conv_wgrad_splits, py::arg("M"), py::arg("Kout"), py::arg("TC"),
        py::arg("ws_cap"), py::arg("taps") = 1);
  m.def("conv_wgrad_halo_splits", [](std::vector<int> geom, std::vector<int> dh, std::vector<int> dw) {
    if (geom.size() != 10) throw std::runtime_error("conv_wgrad_halo_splits: geom needs 10 ints");
    return dtf_conv_wgrad_halo_splits(geom[0], geom[1], geom[2], geom[3], geom[4], geom[5],
                                      geom[8], geom[6], geom[7], make_taps<TapTableW>(dh, dw));
  });
  m.def("wgrad_set_halo", &dtf_wgrad_set_halo);
  m.def("wgrad_set_stem", &dtf_wgrad_set_stem);
  m.def("wgrad_stem_dz_splits", &dtf_wgrad_stem_dz_splits);
  m.def("conv_wgrad_stem_dz", [](uintptr_t x, uintptr_t dp, uintptr_t arg, uintptr_t xbn,
                                 uintptr_t ca, uintptr_t cb, uintptr_t cc, uintptr_t fsc,
                                 uintptr_t fsh, uintptr_t dw, uintptr_t ws, int N, int acc,
                                 uintptr_t st) {
    dtf_conv_wgrad_stem_dz(P<const bf16_t>(x), P<const bf16_t>(dp), P<const uint8_t>(arg),
                           P<const bf16_t>(xbn), P<const float>(ca), P<const float>(cb),
                           P<const float>(cc), P<const float>(fsc), P<const float>(fsh),
                           P<float>(dw), P<float>(ws), N, acc, S(st));
    check_launch("conv_wgrad_stem_dz");
  });
  m.def("wgrad_set_dma_mode", &dtf_wgrad_set_dma_mode);
  m.def("wgrad_set_pipe", &dtf_wgrad_set_pipe);
  m.def("wgrad_set_pp", &dtf_wgrad_set_pp);
  m.def("wgrad_set_dense", &dtf_wgrad_set_dense);
  m.def("wgrad_set_direct", &dtf_wgrad_set_direct);
  m.def("wgrad_set_deep", &dtf_wgrad_set_deep);
  m.def("conv_set_halo_stages", &dtf_conv_set_halo_stages);
  m.def("conv_set_gemm", &dtf_conv_set_gemm);
  m.def("bn_set_nt", &dtf_bn_set_nt);
  m.def("bn_set_grid_cap", &dtf_bn_set_grid_cap);
  m.def("bn_set_stats_blocks", &dtf_bn_set_stats_blocks);
  m.def("conv_set_nt", &dtf_conv_set_nt);
  m.def("gemm_set_nt", &dtf_gemm_set_nt);
  m.def("gemm_set_dbg", &dtf_gemm_set_dbg);
  m.def("gemm_set_stream", &dtf_gemm_set_stream);
  m.def("gemm_stream_ok", &dtf_gemm_stream_ok);
  m.def("gemm_stream_probe", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int probe,
                                uintptr_t stream) {
    dtf_gemm_stream_probe(P<bf16_t>(a), P<bf16_t>(b), P<bf16_t>(c), M, N, probe, S(stream));
    check_launch("gemm_stream_probe");
  });
  m.def("gemm_stream_pre", [](uintptr_t x, uintptr_t b, uintptr_t c, int M, int N, int K,
                              uintptr_t sc, uintptr_t sh, uintptr_t y, uintptr_t stats,
                              uintptr_t stream, int nostore) {
    dtf_gemm_stream_pre(P<bf16_t>(x), P<bf16_t>(b), P<bf16_t>(c), M, N, K, P<float>(sc),
                        P<float>(sh), P<bf16_t>(y), P<float>(stats), S(stream), nostore);
    check_launch("gemm_stream_pre");
  }, py::arg("x"), py::arg("b"), py::arg("c"), py::arg("M"), py::arg("N"), py::arg("K"),
     py::arg("sc"), py::arg("sh"), py::arg("y"), py::arg("stats"), py::arg("stream"),
     py::arg("nostore") = 0);
  m.def("gemm_stream_apply", [](uintptr_t a, uintptr_t w, uintptr_t y, int M, int N, int K,
                                uintptr_t res, uintptr_t sc, uintptr_t sh, uintptr_t mask,
                                uintptr_t stream) {
    dtf_gemm_stream_apply(P<bf16_t>(a), P<bf16_t>(w), P<bf16_t>(y), M, N, K, P<bf16_t>(res),
                          P<float>(sc), P<float>(sh), P<uint8_t>(mask), S(stream));
    check_launch("gemm_stream_apply");
  });
  m.def("gemm_stream_bnb", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K, int lda,
                              int ldb, int ldc, uintptr_t cin, uintptr_t acc_src, uintptr_t acc_mask,
                              uintptr_t bx, uintptr_t mean, uintptr_t inv, uintptr_t sc,
                              uintptr_t sh, uintptr_t bmask, int kind, uintptr_t part,
                              uintptr_t stream, uintptr_t y2, uintptr_t w3, int k3) {
    dtf_gemm_stream_bnb(P<bf16_t>(a), P<bf16_t>(b), P<bf16_t>(c), M, N, K, lda, ldb, ldc,
                        P<bf16_t>(cin), P<bf16_t>(acc_src), P<uint8_t>(acc_mask), P<bf16_t>(bx),
                        P<float>(mean), P<float>(inv), P<float>(sc), P<float>(sh),
                        P<uint8_t>(bmask), kind, P<float>(part), 0, S(stream), P<bf16_t>(y2),
                        P<bf16_t>(w3), k3);
    check_launch("gemm_stream_bnb");
  }, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("M"), py::arg("N"), py::arg("K"),
     py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("cin"), py::arg("acc_src"),
     py::arg("acc_mask"), py::arg("bx"), py::arg("mean"), py::arg("inv"), py::arg("sc"),
     py::arg("sh"), py::arg("bmask"), py::arg("kind"), py::arg("part"), py::arg("stream"),
     py::arg("y2") = 0, py::arg("w3") = 0, py::arg("k3") = 0);
  m.def("gemm_stream_bnb_dual", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K,
                                   int lda, int ldb, int ldc, uintptr_t cin, uintptr_t acc_src,
                                   uintptr_t acc_mask, uintptr_t bx, uintptr_t mean, uintptr_t inv,
                                   uintptr_t bmask, uintptr_t part, uintptr_t bxp, uintptr_t meanp,
                                   uintptr_t invp, uintptr_t part_p, uintptr_t stream) {
    dtf_gemm_stream_bnb_dual(P<bf16_t>(a), P<bf16_t>(b), P<bf16_t>(c), M, N, K, lda, ldb, ldc,
                             P<bf16_t>(cin), P<bf16_t>(acc_src), P<uint8_t>(acc_mask),
                             P<bf16_t>(bx), P<float>(mean), P<float>(inv), P<uint8_t>(bmask),
                             P<float>(part), P<bf16_t>(bxp), P<float>(meanp), P<float>(invp),
                             P<float>(part_p), S(stream));
    check_launch("gemm_stream_bnb_dual");
  });
  m.def("gemm_set_stagger", &dtf_gemm_set_stagger);
  m.def("gemm_set_group", &dtf_gemm_set_group);
  m.def("wgrad_get_pipe", &dtf_wgrad_get_pipe);
  m.def("lds_probe", [](int bytes, int blocks, uintptr_t errors, int spin, uintptr_t st) {
    dtf_lds_probe(bytes, blocks, P<int>(errors), spin, S(st));
    check_launch("lds_probe");
  });
  m.def("max_dynamic_lds", &dtf_max_dynamic_lds);

  // ---- transformer (BERT) kernels
  m.def("ln_fwd", [](uintptr_t a, uintptr_t bias, uintptr_t res, uintptr_t gamma, uintptr_t beta,
                     uintptr_t y, uintptr_t s, uintptr_t mean, uintptr_t rstd, int M, int H,
                     float eps, float p_pre, uint32_t seed_pre, float p_post, uint32_t seed_post,
                     uintptr_t ids, uintptr_t tt, uintptr_t word, uintptr_t pos, uintptr_t type,
                     int S_, uintptr_t st) {
    dtf_ln_fwd(P<const bf16_t>(a), P<const float>(bias), P<const bf16_t>(res),
               P<const float>(gamma), P<const float>(beta), P<bf16_t>(y), P<bf16_t>(s),
               P<float>(mean), P<float>(rstd), M, H, eps, p_pre, seed_pre, p_post, seed_post,
               P<const int64_t>(ids), P<const int64_t>(tt), P<const bf16_t>(word),
               P<const bf16_t>(pos), P<const bf16_t>(type), S_, S(st));
    check_launch("ln_fwd");
  });
  m.def("ln_bwd_blocks", &dtf_ln_bwd_blocks);
  m.def("ln_bwd", [](uintptr_t dy, uintptr_t s, uintptr_t mean, uintptr_t rstd, uintptr_t gamma,
                     uintptr_t ds, uintptr_t da, uintptr_t part, uintptr_t dgamma,
                     uintptr_t dbeta, uintptr_t dbias, int M, int H, float p_pre,
                     uint32_t seed_pre, float p_post, uint32_t seed_post, uintptr_t st,
                     int accumulate) {
    dtf_ln_bwd(P<const bf16_t>(dy), P<const bf16_t>(s), P<const float>(mean),
               P<const float>(rstd), P<const float>(gamma), P<bf16_t>(ds), P<bf16_t>(da),
               P<float>(part), P<float>(dgamma), P<float>(dbeta), P<float>(dbias), M, H, p_pre,
               seed_pre, p_post, seed_post, S(st), accumulate);
    check_launch("ln_bwd");
  }, py::arg("dy"), py::arg("s"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"),
     py::arg("ds"), py::arg("da"), py::arg("part"), py::arg("dgamma"), py::arg("dbeta"),
     py::arg("dbias"), py::arg("M"), py::arg("H"), py::arg("p_pre"), py::arg("seed_pre"),
     py::arg("p_post"), py::arg("seed_post"), py::arg("stream"), py::arg("accumulate") = 0);
  m.def("bias_gelu_fwd", [](uintptr_t a, uintptr_t bias, uintptr_t y, long M, int N,
                            uintptr_t st) {
    dtf_bias_gelu_fwd(P<const bf16_t>(a), P<const float>(bias), P<bf16_t>(y), M, N, S(st));
    check_launch("bias_gelu_fwd");
  });
  m.def("bias_gelu_bwd_blocks", &dtf_bias_gelu_bwd_blocks);
  m.def("bf16_col_sum_ws_floats", &dtf_bf16_col_sum_ws_floats);
  m.def("bf16_col_sum", [](uintptr_t x, int T, int N, uintptr_t ws, uintptr_t out, int accumulate,
                           uintptr_t stream) {
    dtf_bf16_col_sum(P<const bf16_t>(x), T, N, P<float>(ws), P<float>(out), accumulate, S(stream));
  });
  m.def("ln_set_wide", &dtf_ln_set_wide);
  m.def("conv1x1_bwd_ok", &dtf_conv1x1_bwd_ok);
  m.def("conv1x1_bwd_blocks", &dtf_conv1x1_bwd_blocks);
  m.def("conv1x1_bwd_set_grid", &dtf_conv1x1_bwd_set_grid);
  m.def("conv1x1_bwd_set_w16", &dtf_conv1x1_bwd_set_w16);
  m.def("conv1x1_bwd_lazy_ok", &dtf_conv1x1_bwd_lazy_ok);
  m.def("conv1x1_bwd_lazy_blocks", &dtf_conv1x1_bwd_lazy_blocks);
  m.def("conv1x1_bwd_lazy", [](uintptr_t dy3, uintptr_t x3, uintptr_t mask, uintptr_t cA,
                               uintptr_t cB, uintptr_t cC, uintptr_t wt, uintptr_t y, uintptr_t x,
                               uintptr_t mean, uintptr_t inv, uintptr_t sc, uintptr_t sh,
                               uintptr_t dy, uintptr_t wpart, uintptr_t bpart, int M, int C, int K,
                               uintptr_t w, uintptr_t stream) {
    dtf_conv1x1_bwd_lazy(P<bf16_t>(dy3), P<bf16_t>(x3), P<uint8_t>(mask), P<float>(cA),
                         P<float>(cB), P<float>(cC), P<bf16_t>(wt), P<bf16_t>(y), P<bf16_t>(x),
                         P<float>(mean), P<float>(inv), P<float>(sc), P<float>(sh), P<bf16_t>(dy),
                         P<float>(wpart), P<float>(bpart), M, C, K, P<bf16_t>(w), S(stream));
    check_launch("conv1x1_bwd_lazy");
  });
  m.def("conv1x1_bwd", [](uintptr_t dout, uintptr_t wt, uintptr_t y, uintptr_t x, uintptr_t mean,
                          uintptr_t inv, uintptr_t sc, uintptr_t sh, uintptr_t dy, uintptr_t wpart,
                          uintptr_t bpart, int M, int C, int K, uintptr_t stream) {
    dtf_conv1x1_bwd(P<bf16_t>(dout), P<bf16_t>(wt), P<bf16_t>(y), P<bf16_t>(x), P<float>(mean),
                    P<float>(inv), P<float>(sc), P<float>(sh), P<bf16_t>(dy), P<float>(wpart),
                    P<float>(bpart), M, C, K, S(stream));
    check_launch("conv1x1_bwd");
  });
  m.def("slab_reduce", [](uintptr_t ws, uintptr_t out, long n, int nsplit, int accumulate,
                          uintptr_t stream) {
    dtf_slab_reduce(P<const float>(ws), P<float>(out), n, nsplit, accumulate, S(stream));
  });
  m.def("bias_gelu_bwd", [](uintptr_t dy, uintptr_t a, uintptr_t bias, uintptr_t da,
                            uintptr_t part, uintptr_t dbias, int M, int N, uintptr_t st,
                            int accumulate) {
    dtf_bias_gelu_bwd(P<const bf16_t>(dy), P<const bf16_t>(a), P<const float>(bias),
                      P<bf16_t>(da), P<float>(part), P<float>(dbias), M, N, S(st), accumulate);
    check_launch("bias_gelu_bwd");
  }, py::arg("dy"), py::arg("a"), py::arg("bias"), py::arg("da"), py::arg("part"),
     py::arg("dbias"), py::arg("M"), py::arg("N"), py::arg("stream"), py::arg("accumulate") = 0);
  m.def("attn_fwd", [](uintptr_t qkv, uintptr_t mask, uintptr_t out, uintptr_t lse, int B, int S_,
                       int H, float scale, float p, uint32_t seed, uintptr_t st, uintptr_t keep) {
    dtf_attn_fwd(P<const bf16_t>(qkv), P<const float>(mask), P<bf16_t>(out), P<float>(lse), B,
                 S_, H, scale, p, seed, S(st), P<uint32_t>(keep));
    check_launch("attn_fwd");
  }, py::arg("qkv"), py::arg("mask"), py::arg("out"), py::arg("lse"), py::arg("B"), py::arg("S"),
     py::arg("H"), py::arg("scale"), py::arg("p"), py::arg("seed"), py::arg("st"),
     py::arg("keep") = 0);
  m.def("attn_keep_words", &dtf_attn_keep_words);
  m.def("attn_set_keep", &dtf_attn_set_keep);
  m.def("attn_bwd", [](uintptr_t qkv, uintptr_t mask, uintptr_t out, uintptr_t dout,
                       uintptr_t lse, uintptr_t delta, uintptr_t dqkv, int B, int S_, int H,
                       float scale, float p, uint32_t seed, uintptr_t st, uintptr_t colpart,
                       uintptr_t keep) {
    dtf_attn_bwd(P<const bf16_t>(qkv), P<const float>(mask), P<const bf16_t>(out),
                 P<const bf16_t>(dout), P<const float>(lse), P<float>(delta), P<bf16_t>(dqkv), B,
                 S_, H, scale, p, seed, S(st), P<float>(colpart), P<const uint32_t>(keep));
    check_launch("attn_bwd");
  }, py::arg("qkv"), py::arg("mask"), py::arg("out"), py::arg("dout"), py::arg("lse"),
     py::arg("delta"), py::arg("dqkv"), py::arg("B"), py::arg("S"), py::arg("H"),
     py::arg("scale"), py::arg("p"), py::arg("seed"), py::arg("st"), py::arg("colpart") = 0,
     py::arg("keep") = 0);
  m.def("attn_bwd_fused", &dtf_attn_bwd_fused);
  m.def("attn_set_wide", &dtf_attn_set_wide);
  m.def("attn_set_fused", &dtf_attn_set_fused);
  m.def("pos_type_grad_ws_floats", &dtf_pos_type_grad_ws_floats);
  m.def("pos_type_grad", [](uintptr_t ds, uintptr_t tt, int B, int S_, int H, int NT,
                            uintptr_t dpos, uintptr_t dtyp, uintptr_t ws, uintptr_t st) {
    dtf_pos_type_grad(P<const bf16_t>(ds), P<const int64_t>(tt), B, S_, H, NT, P<float>(dpos),
                      P<float>(dtyp), P<float>(ws), S(st));
    check_launch("pos_type_grad");
  });
  m.def("segment_sum", [](uintptr_t sorted_ids, uintptr_t perm, uintptr_t src, uintptr_t out,
                          int T, int H, uintptr_t st) {
    dtf_segment_sum(P<const int64_t>(sorted_ids), P<const int64_t>(perm), P<const bf16_t>(src),
                    P<float>(out), T, H, S(st));
    check_launch("segment_sum");
  });
  m.def("mlm_xent", [](uintptr_t logits, uintptr_t labels, uintptr_t weights, uintptr_t denom,
                       int N, int V, int ld, uintptr_t loss_rows, uintptr_t grad, uintptr_t st) {
    dtf_mlm_xent(P<const bf16_t>(logits), P<const int64_t>(labels), P<const float>(weights),
                 P<const float>(denom), N, V, ld, P<float>(loss_rows), P<bf16_t>(grad), S(st));
    check_launch("mlm_xent");
  });
}
