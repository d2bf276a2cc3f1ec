// PyTorch-ROCm custom operators over the C ABI of libmog_air.so
// (include/mog_air.h): TORCH_LIBRARY_FRAGMENT(mog_air) schemas with HIP
// (dispatch key CUDA on ROCm) implementations, so the Python host drives every
// hot-path launch through torch.ops.mog_air.*  -- the AIR
// model (air/air_model.py) and the AIR-ASR model
// (air/air_number_bbox_location.py) alike.  Each op takes device tensors (or
// views: a tensor's data_ptr is the matrix origin, leading dimensions are
// explicit) and plain scalars, launches on torch's current HIP stream of the
// operands' device, and raises (c10::Error -> RuntimeError) when an operand is
// on the wrong device, has the wrong dtype or is too small for the extent the
// launch touches, or when the C ABI rejects an argument.  There is no CPU
// kernel: a CPU tensor finds no implementation and fails loudly.  Every
// argument an op writes carries a (x!) alias annotation in its schema.
//
// The ops are the launch-level (mutating, "out=") form the models schedule
// their forward / backward with; differentiable functional ops built on them
// live in mog_air/torch_ops.py.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "mog_air.h"

namespace {

using at::ScalarType;
using at::Tensor;
using c10::optional;
using std::vector;

constexpr ScalarType F32 = at::kFloat, BF16 = at::kBFloat16, I32 = at::kInt;

void check(int rc, const char* name) {
  TORCH_CHECK(rc == 0, "mog_air::", name, " failed: ",
              rc == MOG_ERR_INVALID ? "invalid argument" : "HIP error ", rc);
}

// Operand validation: every tensor on the op's device (the first checked
// operand fixes it), of the dtype the C ABI reads, and holding at least
// `extent` elements from its data_ptr (the span the launch reads or writes).
struct Op {
  const char* name;
  c10::optional<c10::Device> dev;
  explicit Op(const char* n) : name(n) {}
  void* need(const Tensor& t, ScalarType st, int64_t extent, const char* arg) {
    TORCH_CHECK(t.defined(), name, ": ", arg, " is undefined");
    TORCH_CHECK(t.is_cuda(), name, ": ", arg,
                " must be a HIP device tensor (there is no CPU implementation)");
    if (!dev) dev = t.device();
    TORCH_CHECK(t.device() == *dev, name, ": ", arg, " is on ", t.device(), ", the op on ", *dev);
    TORCH_CHECK(t.scalar_type() == st, name, ": ", arg, " must be ", st, ", got ",
                t.scalar_type());
    if (extent > 0) {
      const int64_t avail =
          (int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
      TORCH_CHECK(extent <= avail, name, ": ", arg, " holds ", avail,
                  " elements from its origin, the launch touches ", extent);
    }
    return t.data_ptr();
  }
  void* need(const optional<Tensor>& t, ScalarType st, int64_t extent, const char* arg) {
    return t.has_value() && t->defined() ? need(*t, st, extent, arg) : nullptr;
  }
  float* f(const Tensor& t, int64_t extent, const char* arg) {
    return static_cast<float*>(need(t, F32, extent, arg));
  }
  float* f(const optional<Tensor>& t, int64_t extent, const char* arg) {
    return static_cast<float*>(need(t, F32, extent, arg));
  }
  int* i(const Tensor& t, int64_t extent, const char* arg) {
    return static_cast<int*>(need(t, I32, extent, arg));
  }
  int* i(const optional<Tensor>& t, int64_t extent, const char* arg) {
    return static_cast<int*>(need(t, I32, extent, arg));
  }
  // device pointer arrays of tensor lists (None entries -> NULL)
  vector<void*> list(at::TensorList ts, ScalarType st, int64_t extent, const char* arg) {
    vector<void*> v;
    for (const auto& t : ts) v.push_back(need(t, st, extent, arg));
    return v;
  }
  vector<void*> list(const c10::List<optional<Tensor>>& ts, ScalarType st, int64_t extent,
                     const char* arg) {
    vector<void*> v;
    for (size_t k = 0; k < ts.size(); ++k)
      v.push_back(need(static_cast<optional<Tensor>>(ts[k]), st, extent, arg));
    return v;
  }
  // the current HIP stream of the op's device (set by the guard)
  void* stream() {
    TORCH_CHECK(dev.has_value(), name, ": no device operand");
    return c10::hip::getCurrentHIPStream(dev->index()).stream();
  }
};

// elements spanned by a rows x cols matrix with leading dimension ld
int64_t mat(int64_t rows, int64_t cols, int64_t ld) {
  return rows <= 0 || cols <= 0 ? 0 : (rows - 1) * ld + cols;
}

template <class T>
const T* const* arr(const vector<void*>& v) {
  return v.empty() ? nullptr : reinterpret_cast<const T* const*>(v.data());
}
template <class T>
T* const* marr(const vector<void*>& v) {
  return v.empty() ? nullptr : reinterpret_cast<T* const*>(v.data());
}

#define GUARD(op) const c10::hip::HIPGuardMasqueradingAsCUDA guard_(*op.dev)

// ---------------------------------------------------------------- GEMMs ----
void gemm_f32_(at::TensorList A, at::TensorList B, at::TensorList C,
               const c10::List<optional<Tensor>>& bias, const c10::List<optional<Tensor>>& Cin,
               const c10::List<optional<Tensor>>& Cpre, const c10::List<optional<Tensor>>& aux,
               const c10::List<optional<Tensor>>& colsum, int64_t M, int64_t N, int64_t K,
               int64_t lda, int64_t ldb, int64_t ldc, int64_t ldaux, bool transA, bool transB,
               int64_t epi, double aux_scale, int64_t splitk) {
  Op o("gemm_f32_");
  auto c = o.list(C, F32, mat(M, N, ldc), "C");
  auto a = o.list(A, F32, transA ? mat(K, M, lda) : mat(M, K, lda), "A");
  auto b = o.list(B, F32, transB ? mat(N, K, ldb) : mat(K, N, ldb), "B");
  auto bi = o.list(bias, F32, N, "bias"), ci = o.list(Cin, F32, mat(M, N, ldc), "Cin");
  auto cp = o.list(Cpre, F32, mat(M, N, ldc), "Cpre"), ax = o.list(aux, F32, mat(M, N, ldaux), "aux");
  auto cs = o.list(colsum, F32, N, "colsum");
  GUARD(o);
  check(mog_gemm_f32((int)c.size(), arr<float>(a), arr<float>(b), marr<float>(c), arr<float>(bi),
                     arr<float>(ci), marr<float>(cp), arr<float>(ax), marr<float>(cs), M, N, K, lda,
                     ldb, ldc, ldaux, transA, transB, epi, (float)aux_scale, splitk, o.stream()),
        o.name);
}

void gemm_f32_sigmoid_philox_(const Tensor& A, const Tensor& B, Tensor C,
                              const optional<Tensor>& bias, int64_t M, int64_t N, int64_t K,
                              int64_t lda, int64_t ldb, int64_t ldc, double scale, int64_t seed,
                              int64_t offset) {
  Op o("gemm_f32_sigmoid_philox_");
  float* c = o.f(C, mat(M, N, ldc), "C");
  float* a = o.f(A, mat(M, K, lda), "A");
  float* b = o.f(B, mat(K, N, ldb), "B");
  float* bi = o.f(bias, N, "bias");
  GUARD(o);
  check(mog_gemm_f32_sigmoid_philox(a, b, c, bi, M, N, K, lda, ldb, ldc, (float)scale,
                                    (unsigned long long)seed, (unsigned long long)offset,
                                    o.stream()),
        o.name);
}

void gemm_f32_kseg_(at::TensorList A, at::TensorList B, Tensor C, const optional<Tensor>& bias,
                    const optional<Tensor>& Cin, int64_t M, int64_t N, int64_t kseg, int64_t lda,
                    int64_t ldb, int64_t ldc, bool transA, bool transB, int64_t epi) {
  Op o("gemm_f32_kseg_");
  float* c = o.f(C, mat(M, N, ldc), "C");
  auto a = o.list(A, F32, transA ? mat(kseg, M, lda) : mat(M, kseg, lda), "A");
  auto b = o.list(B, F32, transB ? mat(N, kseg, ldb) : mat(kseg, N, ldb), "B");
  TORCH_CHECK(a.size() == b.size(), o.name, ": as many A as B segments");
  float* bi = o.f(bias, N, "bias");
  float* ci = o.f(Cin, mat(M, N, ldc), "Cin");
  GUARD(o);
  check(mog_gemm_f32_kseg((int)a.size(), arr<float>(a), arr<float>(b), c, bi, ci, M, N, kseg, lda,
                          ldb, ldc, transA, transB, epi, o.stream()),
        o.name);
}

void gemm_f32_kseg_group_(at::TensorList A, at::TensorList B, at::TensorList C,
                          const c10::List<optional<Tensor>>& Cin, at::IntArrayRef nseg, int64_t M,
                          int64_t N, int64_t kseg, int64_t lda, int64_t ldb, int64_t ldc,
                          bool transB) {
  Op o("gemm_f32_kseg_group_");
  auto c = o.list(C, F32, mat(M, N, ldc), "C");
  auto a = o.list(A, F32, mat(M, kseg, lda), "A");
  auto b = o.list(B, F32, transB ? mat(N, kseg, ldb) : mat(kseg, N, ldb), "B");
  auto ci = o.list(Cin, F32, mat(M, N, ldc), "Cin");
  TORCH_CHECK(nseg.size() == c.size() && ci.size() == c.size(), o.name,
              ": nseg / Cin / C of one length");
  int64_t tot = 0;
  std::vector<int> ns;
  for (auto n : nseg) {
    ns.push_back((int)n);
    tot += n;
  }
  TORCH_CHECK(a.size() == (size_t)tot && b.size() == (size_t)tot, o.name,
              ": sum(nseg) A and B segments");
  GUARD(o);
  check(mog_gemm_f32_kseg_group((int)c.size(), ns.data(), arr<float>(a), arr<float>(b),
                                marr<float>(c), arr<float>(ci), M, N,
                                kseg, lda, ldb, ldc, transB, o.stream()),
        o.name);
}

void gemm_bf16_(at::TensorList A, at::TensorList B, at::TensorList C,
                const c10::List<optional<Tensor>>& bias, const c10::List<optional<Tensor>>& Cin,
                const c10::List<optional<Tensor>>& aux, const c10::List<optional<Tensor>>& colsum,
                int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                int64_t ldaux, bool tn, int64_t epi, double aux_scale, int64_t splitk) {
  Op o("gemm_bf16_");
  TORCH_CHECK(C.size() > 0, o.name, ": no output");
  const bool out_bf16 = C[0].scalar_type() == BF16;
  auto c = o.list(C, out_bf16 ? BF16 : F32, mat(M, N, ldc), "C");
  auto a = o.list(A, BF16, tn ? mat(K, M, lda) : mat(M, K, lda), "A");
  auto b = o.list(B, BF16, tn ? mat(K, N, ldb) : mat(N, K, ldb), "B");
  auto bi = o.list(bias, F32, N, "bias"), ci = o.list(Cin, F32, mat(M, N, ldc), "Cin");
  // aux: the noise (epi 2, fp32) or the softplus output (epi 3, bf16)
  auto ax = o.list(aux, epi == 3 ? BF16 : F32, mat(M, N, ldaux), "aux");
  auto cs = o.list(colsum, F32, N, "colsum");
  GUARD(o);
  check(mog_gemm_bf16((int)c.size(), arr<void>(a), arr<void>(b), marr<void>(c), arr<float>(bi),
                      arr<float>(ci), arr<void>(ax), marr<float>(cs), M, N, K, lda, ldb, ldc,
                      ldaux, tn, epi, out_bf16, (float)aux_scale, splitk, o.stream()),
        o.name);
}

void cvt_bf16_batch_(at::TensorList src, at::TensorList dst, at::IntArrayRef dims) {
  Op o("cvt_bf16_batch_");
  TORCH_CHECK(dims.size() == 7 * src.size() && src.size() == dst.size(),
              o.name, ": 7 dims per job");
  vector<void*> s, d;
  vector<int> di(dims.begin(), dims.end());
  for (size_t j = 0; j < src.size(); ++j) {
    const int* q = &di[7 * j];  // src_rows, src_cols, ld_src, rows, cols, ld_dst, transpose
    s.push_back(o.need(src[j], F32, mat(q[0], q[1], q[2]), "src"));
    d.push_back(o.need(dst[j], BF16, q[6] == 2 ? (int64_t)q[3] * q[4] : mat(q[3], q[4], q[5]),
                       "dst"));
  }
  GUARD(o);
  check(mog_cvt_bf16_batch((int)s.size(), arr<float>(s), marr<void>(d), di.data(), o.stream()),
        o.name);
}

// ------------------------------------------------------------------ STN ----
void stn_forward_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win, const Tensor& theta,
                  int64_t Hout, int64_t Wout, Tensor out, const optional<Tensor>& z,
                  const optional<Tensor>& mask, int64_t mode, int64_t u_period) {
  Op o("stn_forward_");
  TORCH_CHECK(u_period >= 0, o.name, ": u_period >= 0");
  void* po = o.need(out, mode == 2 ? BF16 : F32, N * Hout * Wout, "out");
  float* pu = o.f(U, (u_period > 0 ? std::min(u_period, N) : N) * Hin * Win, "U");
  float* pt = o.f(theta, N * 6, "theta");
  float* pz = o.f(z, N, "z");
  float* pm = o.f(mask, N, "mask");
  GUARD(o);
  check(mog_stn_forward_periodic(pu, u_period, N, Hin, Win, pt, Hout, Wout, po, pz, pm, mode,
                                 o.stream()),
        o.name);
}

void stn_backward_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win, const Tensor& theta,
                   int64_t Hout, int64_t Wout, const Tensor& G, const optional<Tensor>& gscale,
                   const optional<Tensor>& dU, const optional<Tensor>& dtheta,
                   const optional<Tensor>& dot, int64_t u_period, int64_t g_period) {
  Op o("stn_backward_");
  float* pu = o.f(U, (u_period > 0 ? u_period : N) * Hin * Win, "U");
  float* pt = o.f(theta, N * 6, "theta");
  float* pg = o.f(G, (g_period > 0 ? g_period : N) * Hout * Wout, "G");
  float* ps = o.f(gscale, N, "gscale");
  float* pdu = o.f(dU, N * Hin * Win, "dU");
  float* pdt = o.f(dtheta, N * 6, "dtheta");
  float* pd = o.f(dot, N, "dot");
  GUARD(o);
  check(mog_stn_backward(pu, N, Hin, Win, pt, Hout, Wout, pg, ps, pdu, pdt, pd, u_period,
                         g_period, o.stream()),
        o.name);
}

void stn_backward_sigmoid_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win,
                           const Tensor& theta, int64_t Hout, int64_t Wout, const Tensor& G,
                           const optional<Tensor>& gscale, Tensor dm,
                           const optional<Tensor>& dtheta, const optional<Tensor>& dot,
                           int64_t g_period) {
  // dm bf16 (configs[1]) or fp32 (reference precision)
  Op o("stn_backward_sigmoid_");
  const bool bf = dm.scalar_type() == BF16;
  void* pdm = o.need(dm, bf ? BF16 : F32, N * Hin * Win, "dm");
  float* pu = o.f(U, N * Hin * Win, "U");
  float* pt = o.f(theta, N * 6, "theta");
  float* pg = o.f(G, (g_period > 0 ? g_period : N) * Hout * Wout, "G");
  float* ps = o.f(gscale, N, "gscale");
  float* pdt = o.f(dtheta, N * 6, "dtheta");
  float* pd = o.f(dot, N, "dot");
  GUARD(o);
  if (bf)
    check(mog_stn_backward_sigmoid_bf16(pu, N, Hin, Win, pt, Hout, Wout, pg, ps, pdm, pdt, pd, 0,
                                        g_period, o.stream()),
          o.name);
  else
    check(mog_stn_backward_sigmoid_f32(pu, N, Hin, Win, pt, Hout, Wout, pg, ps,
                                       static_cast<float*>(pdm), pdt, pd, 0, g_period,
                                       o.stream()),
          o.name);
}

void stn_write_parts_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win, const Tensor& theta,
                      int64_t Hout, int64_t Wout, const Tensor& z, const Tensor& mask, Tensor parts,
                      Tensor part_rows) {
  Op o("stn_write_parts_");
  float* pp = o.f(parts, N * Hout * Wout, "parts");
  int* pr = o.i(part_rows, N, "part_rows");
  float* pu = o.f(U, N * Hin * Win, "U");
  float* pt = o.f(theta, N * 6, "theta");
  float* pz = o.f(z, N, "z");
  float* pm = o.f(mask, N, "mask");
  GUARD(o);
  check(mog_stn_write_parts(pu, N, Hin, Win, pt, Hout, Wout, pz, pm, pp, pr, o.stream()), o.name);
}

// ----------------------------------------------------------------- LSTM ----
void lstm_cell_forward_(const Tensor& G, const optional<Tensor>& bias,
                        const optional<Tensor>& c_prev, Tensor c_out, Tensor h_out, int64_t B,
                        int64_t H) {
  Op o("lstm_cell_forward_");
  float* pc = o.f(c_out, B * H, "c_out");
  float* ph = o.f(h_out, B * H, "h_out");
  float* pg = o.f(G, B * 4 * H, "G");
  float* pb = o.f(bias, 4 * H, "bias");
  float* pp = o.f(c_prev, B * H, "c_prev");
  GUARD(o);
  check(mog_lstm_cell_forward(pg, pb, pp, pc, ph, B, H, o.stream()), o.name);
}

void lstm_cell_backward_(const Tensor& G, const optional<Tensor>& bias,
                         const optional<Tensor>& c_prev, const Tensor& c_cur, const Tensor& dh,
                         const optional<Tensor>& dc, Tensor dG, Tensor dc_prev,
                         const optional<Tensor>& dGsum, int64_t B, int64_t H) {
  Op o("lstm_cell_backward_");
  float* pdg = o.f(dG, B * 4 * H, "dG");
  float* pdcp = o.f(dc_prev, B * H, "dc_prev");
  float* pg = o.f(G, B * 4 * H, "G");
  float* pb = o.f(bias, 4 * H, "bias");
  float* pcp = o.f(c_prev, B * H, "c_prev");
  float* pcc = o.f(c_cur, B * H, "c_cur");
  float* pdh = o.f(dh, B * H, "dh");
  float* pdc = o.f(dc, B * H, "dc");
  float* pgs = o.f(dGsum, B * 4 * H, "dGsum");
  GUARD(o);
  check(mog_lstm_cell_backward(pg, pb, pcp, pcc, pdh, pdc, pdg, pdcp, pgs, B, H, o.stream()),
        o.name);
}

// the cell backward summing the K-split parts of the dh GEMM into dh
// (mog_lstm_cell_backward_parts)
void lstm_cell_backward_parts_(const Tensor& G, const optional<Tensor>& bias,
                               const optional<Tensor>& c_prev, const Tensor& c_cur,
                               const Tensor& dh, const Tensor& dh_parts, int64_t nparts,
                               const optional<Tensor>& dc, Tensor dG, Tensor dc_prev,
                               const optional<Tensor>& dGsum, int64_t B, int64_t H) {
  Op o("lstm_cell_backward_parts_");
  float* pdg = o.f(dG, B * 4 * H, "dG");
  float* pdcp = o.f(dc_prev, B * H, "dc_prev");
  float* pg = o.f(G, B * 4 * H, "G");
  float* pb = o.f(bias, 4 * H, "bias");
  float* pcp = o.f(c_prev, B * H, "c_prev");
  float* pcc = o.f(c_cur, B * H, "c_cur");
  float* pdh = o.f(dh, B * H, "dh");
  float* ppt = o.f(dh_parts, nparts * B * H, "dh_parts");
  float* pdc = o.f(dc, B * H, "dc");
  float* pgs = o.f(dGsum, B * 4 * H, "dGsum");
  GUARD(o);
  check(mog_lstm_cell_backward_parts(pg, pb, pcp, pcc, pdh, ppt, (int)nparts, B * H, pdc, pdg,
                                     pdcp, pgs, B, H, o.stream()),
        o.name);
}

// the two cells of one batch in one launch (no bias: both cells' gate GEMMs
// add theirs)
void lstm_cell_forward2_(const Tensor& G0, const optional<Tensor>& c_prev0, Tensor c_out0,
                         Tensor h_out0, const Tensor& G1, const optional<Tensor>& c_prev1,
                         Tensor c_out1, Tensor h_out1, int64_t B, int64_t H) {
  Op o("lstm_cell_forward2_");
  const float* p[10] = {o.f(G0, B * 4 * H, "G0"), nullptr, o.f(c_prev0, B * H, "c_prev0"),
                        o.f(c_out0, B * H, "c_out0"), o.f(h_out0, B * H, "h_out0"),
                        o.f(G1, B * 4 * H, "G1"), nullptr, o.f(c_prev1, B * H, "c_prev1"),
                        o.f(c_out1, B * H, "c_out1"), o.f(h_out1, B * H, "h_out1")};
  GUARD(o);
  check(mog_lstm_cell_forward_pair(p, B, H, o.stream()), o.name);
}

void lstm_cell_backward2_(const Tensor& G0, const optional<Tensor>& c_prev0, const Tensor& c_cur0,
                          const Tensor& dh0, const optional<Tensor>& dc0, Tensor dG0,
                          Tensor dc_prev0, const optional<Tensor>& dGsum0, const Tensor& G1,
                          const optional<Tensor>& c_prev1, const Tensor& c_cur1,
                          const Tensor& dh1, const optional<Tensor>& dc1, Tensor dG1,
                          Tensor dc_prev1, const optional<Tensor>& dGsum1, int64_t B, int64_t H) {
  Op o("lstm_cell_backward2_");
  const float* p[18] = {o.f(G0, B * 4 * H, "G0"),        nullptr,
                        o.f(c_prev0, B * H, "c_prev0"),  o.f(c_cur0, B * H, "c_cur0"),
                        o.f(dh0, B * H, "dh0"),          o.f(dc0, B * H, "dc0"),
                        o.f(dG0, B * 4 * H, "dG0"),      o.f(dc_prev0, B * H, "dc_prev0"),
                        o.f(dGsum0, B * 4 * H, "dGsum0"), o.f(G1, B * 4 * H, "G1"),
                        nullptr,                         o.f(c_prev1, B * H, "c_prev1"),
                        o.f(c_cur1, B * H, "c_cur1"),    o.f(dh1, B * H, "dh1"),
                        o.f(dc1, B * H, "dc1"),          o.f(dG1, B * 4 * H, "dG1"),
                        o.f(dc_prev1, B * H, "dc_prev1"), o.f(dGsum1, B * 4 * H, "dGsum1")};
  GUARD(o);
  check(mog_lstm_cell_backward_pair(p, B, H, o.stream()), o.name);
}

// ------------------------------------------------ heads / concrete / masks ----
void air_step_forward_(int64_t B, int64_t HS, int64_t HZ, int64_t step, bool train,
                       bool use_num_prior, double thr, double temperature, double prior_lo,
                       double prior_bias, double s_pm, double s_pv, double s_plv, double h_pm,
                       double h_pv, double h_plv, at::TensorList hid, at::TensorList w2,
                       at::TensorList b2, const Tensor& eps_scale, const Tensor& eps_shift,
                       const Tensor& u, Tensor stop, Tensor runloss, Tensor digits, Tensor live,
                       Tensor rec, Tensor theta_fwd, Tensor theta_back, Tensor scale, Tensor shift,
                       Tensor zprob, Tensor zkl, Tensor skl, Tensor shkl, Tensor zmask, Tensor zval,
                       Tensor zc, const optional<Tensor>& prior_lo_dev) {
  Op o("air_step_forward_");
  TORCH_CHECK(hid.size() == 5 && w2.size() == 5 && b2.size() == 5, o.name, ": 5 heads");
  float* pst = o.f(stop, B, "stop");
  auto h = o.list(hid, F32, B * HS, "hid"), w = o.list(w2, F32, HS, "w2"),
       b = o.list(b2, F32, 1, "b2");
  float* pes = o.f(eps_scale, B, "eps_scale");
  float* peh = o.f(eps_shift, 2 * B, "eps_shift");
  float* pu = o.f(u, B, "u");
  float* prl = o.f(runloss, B, "runloss");
  int* pd = o.i(digits, B, "digits");
  int* pl = o.i(live, step + 2, "live");
  float* pr = o.f(rec, 17 * B, "rec");
  float* ptf = o.f(theta_fwd, 6 * B, "theta_fwd");
  float* ptb = o.f(theta_back, 6 * B, "theta_back");
  float* psc = o.f(scale, B, "scale");
  float* psh = o.f(shift, 2 * B, "shift");
  float* pzp = o.f(zprob, B, "zprob");
  float* pzk = o.f(zkl, B, "zkl");
  float* psk = o.f(skl, B, "skl");
  float* phk = o.f(shkl, B, "shkl");
  float* pzm = o.f(zmask, B, "zmask");
  float* pzv = o.f(zval, B, "zval");
  float* pzc = o.f(zc, B, "zc");
  float* pplo = o.f(prior_lo_dev, 1, "prior_lo_dev");
  GUARD(o);
  check(mog_air_step_forward(B, HS, HZ, step, train, use_num_prior, thr, temperature, prior_lo,
                             prior_bias, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv, arr<float>(h),
                             arr<float>(w), arr<float>(b), pes, peh, pu, pst, prl, pd, pl, pr, ptf,
                             ptb, psc, psh, pzp, pzk, psk, phk, pzm, pzv, pzc, pplo, o.stream()),
        o.name);
}

// every loop step in one launch (mog_air_step_forward_steps): operands over
// steps * B rows, hid[z] over steps * B rows of HS (HZ for the z_pres head)
void air_step_forward_steps_(int64_t steps, int64_t B, int64_t HS, int64_t HZ, bool train,
                             bool use_num_prior, double thr, double temperature, double prior_lo,
                             at::ArrayRef<double> prior_bias, double s_pm, double s_pv,
                             double s_plv, double h_pm, double h_pv, double h_plv,
                             at::TensorList hid, at::TensorList w2, at::TensorList b2,
                             const Tensor& eps_scale, const Tensor& eps_shift, const Tensor& u,
                             Tensor stop, Tensor digits, Tensor live, Tensor rec,
                             Tensor theta_fwd, Tensor theta_back, Tensor scale, Tensor shift,
                             Tensor zprob, Tensor zkl, Tensor skl, Tensor shkl, Tensor zmask,
                             Tensor zval, Tensor zc, const optional<Tensor>& prior_lo_dev) {
  Op o("air_step_forward_steps_");
  TORCH_CHECK(hid.size() == 5 && w2.size() == 5 && b2.size() == 5, o.name, ": 5 heads");
  TORCH_CHECK(steps >= 1 && steps <= 8 && (int64_t)prior_bias.size() == steps, o.name,
              ": 1 <= steps <= 8 and one prior bias per step");
  TORCH_CHECK(HZ == HS, o.name, ": the heads' hidden rows are one [5, steps * B, HS] layout");
  const int64_t R = steps * B;
  float* pst = o.f(stop, B, "stop");
  auto h = o.list(hid, F32, R * HS, "hid"), w = o.list(w2, F32, HS, "w2"),
       b = o.list(b2, F32, 1, "b2");
  float* pes = o.f(eps_scale, R, "eps_scale");
  float* peh = o.f(eps_shift, 2 * R, "eps_shift");
  float* pu = o.f(u, R, "u");
  int* pd = o.i(digits, B, "digits");
  int* pl = o.i(live, steps + 1, "live");
  float* pr = o.f(rec, 17 * R, "rec");
  float* ptf = o.f(theta_fwd, 6 * R, "theta_fwd");
  float* ptb = o.f(theta_back, 6 * R, "theta_back");
  float* psc = o.f(scale, R, "scale");
  float* psh = o.f(shift, 2 * R, "shift");
  float* pzp = o.f(zprob, R, "zprob");
  float* pzk = o.f(zkl, R, "zkl");
  float* psk = o.f(skl, R, "skl");
  float* phk = o.f(shkl, R, "shkl");
  float* pzm = o.f(zmask, R, "zmask");
  float* pzv = o.f(zval, R, "zval");
  float* pzc = o.f(zc, R, "zc");
  float* pplo = o.f(prior_lo_dev, 1, "prior_lo_dev");
  float pb[8];
  for (int64_t t = 0; t < steps; ++t) pb[t] = (float)prior_bias[t];
  GUARD(o);
  check(mog_air_step_forward_steps(steps, B, HS, HZ, train, use_num_prior, thr, temperature,
                                   prior_lo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv,
                                   arr<float>(h), B * HS, arr<float>(w), arr<float>(b), pes, peh,
                                   pu, pst, pd, pl, pr, ptf, ptb, psc, psh, pzp, pzk, psk, phk,
                                   pzm, pzv, pzc, pplo, o.stream()),
        o.name);
}

void air_step_backward_(int64_t B, int64_t HS, bool train, bool use_num_prior,
                        double temperature, double prior_lo, double prior_bias, double s_pm,
                        double s_pv, double h_pm, double h_pv, double grad_scale,
                        const optional<Tensor>& dloss, const Tensor& rec, const Tensor& eps_scale,
                        const Tensor& eps_shift, const Tensor& dtheta_fwd,
                        const Tensor& dtheta_back, const Tensor& dot, at::TensorList hid,
                        at::TensorList w2, Tensor dout, int64_t dout_hs, Tensor dhid,
                        int64_t dhid_hs, const optional<Tensor>& prior_lo_dev, int64_t steps) {
  Op o("air_step_backward_");
  TORCH_CHECK(hid.size() == 5 && w2.size() == 5, o.name, ": 5 heads");
  TORCH_CHECK(steps >= 1, o.name, ": steps >= 1");
  const int64_t R = steps * B;  // rows of all the launch's steps
  float* pdo = o.f(dout, 4 * dout_hs + 2 * R, "dout");
  float* pdh = o.f(dhid, dhid_hs == HS ? 5 * R * HS : 4 * dhid_hs + R * HS, "dhid");
  auto h = o.list(hid, F32, R * HS, "hid"), w = o.list(w2, F32, HS, "w2");
  float* pl = o.f(dloss, B, "dloss");
  float* pr = o.f(rec, 17 * R, "rec");
  float* pes = o.f(eps_scale, R, "eps_scale");
  float* peh = o.f(eps_shift, 2 * R, "eps_shift");
  float* ptf = o.f(dtheta_fwd, 6 * R, "dtheta_fwd");
  float* ptb = o.f(dtheta_back, 6 * R, "dtheta_back");
  float* pd = o.f(dot, R, "dot");
  float* pplo = o.f(prior_lo_dev, 1, "prior_lo_dev");
  GUARD(o);
  check(mog_air_step_backward_steps(steps, B, HS, train, use_num_prior, temperature, prior_lo,
                                    prior_bias, s_pm, s_pv, h_pm, h_pv, grad_scale, pl, pr, pes,
                                    peh, ptf, ptb, pd, arr<float>(h), arr<float>(w), pdo, dout_hs,
                                    pdh, dhid_hs, pplo, o.stream()),
        o.name);
}

void generation_prior_(int64_t G, int64_t Z, double s_pm, double s_plv, double h_pm,
                       double h_plv, double v_pm, double v_plv, const Tensor& eps_scale,
                       const Tensor& eps_shift, const Tensor& eps_z, Tensor theta_back,
                       Tensor scale, Tensor shift, Tensor z) {
  Op o("generation_prior_");
  float* ptb = o.f(theta_back, 6 * G, "theta_back");
  float* psc = o.f(scale, G, "scale");
  float* psh = o.f(shift, 2 * G, "shift");
  float* pz = o.f(z, G * Z, "z");
  float* pes = o.f(eps_scale, G, "eps_scale");
  float* peh = o.f(eps_shift, 2 * G, "eps_shift");
  float* pez = o.f(eps_z, G * Z, "eps_z");
  GUARD(o);
  check(mog_generation_prior(G, Z, s_pm, s_plv, h_pm, h_plv, v_pm, v_plv, pes, peh, pez, ptb, psc,
                             psh, pz, o.stream()),
        o.name);
}

// ------------------------------------------------------------ glimpse VAE ----
void vae_sample_forward_(int64_t B, int64_t Z, double v_pm, double v_pv, double v_plv,
                         const Tensor& mu, const Tensor& lv, const Tensor& eps, Tensor z,
                         const optional<Tensor>& z_bf16, int64_t ld_zb, const Tensor& act,
                         const optional<Tensor>& runloss, Tensor vkl) {
  Op o("vae_sample_forward_");
  float* pz = o.f(z, B * Z, "z");
  void* pzb = o.need(z_bf16, BF16, mat(B, Z, ld_zb), "z_bf16");
  float* pm = o.f(mu, B * Z, "mu");
  float* pl = o.f(lv, B * Z, "lv");
  float* pe = o.f(eps, B * Z, "eps");
  float* pa = o.f(act, B, "act");
  float* prl = o.f(runloss, B, "runloss");
  float* pk = o.f(vkl, B, "vkl");
  GUARD(o);
  check(mog_vae_sample_forward(B, Z, v_pm, v_pv, v_plv, pm, pl, pe, pz, pzb, ld_zb, pa, prl, pk,
                               o.stream()),
        o.name);
}

void air_runloss_(int64_t T, int64_t B, Tensor rec, int64_t rec_step_stride, const Tensor& skl,
                  const Tensor& shkl, const Tensor& vkl, Tensor runloss,
                  const optional<Tensor>& live) {
  Op o("air_runloss_");
  float* prl = o.f(runloss, B, "runloss");
  float* pr = o.f(rec, (T - 1) * rec_step_stride + 17 * B, "rec");
  float* ps = o.f(skl, T * B, "skl");
  float* ph = o.f(shkl, T * B, "shkl");
  float* pv = o.f(vkl, T * B, "vkl");
  int* pl = live.has_value() ? o.i(*live, T, "live") : nullptr;
  GUARD(o);
  check(mog_air_runloss(T, B, pr, rec_step_stride, ps, ph, pv, prl, pl, o.stream()), o.name);
}

void vae_sample_backward_(int64_t B, int64_t Z, double v_pm, double v_pv, double grad_scale,
                          const Tensor& mu, const Tensor& lv, const Tensor& eps, const Tensor& dz,
                          const Tensor& act, const optional<Tensor>& dmu,
                          const optional<Tensor>& dlv, const optional<Tensor>& dmu_bf16,
                          const optional<Tensor>& dlv_bf16, int64_t ld_b) {
  Op o("vae_sample_backward_");
  float* pm = o.f(mu, B * Z, "mu");
  float* pl = o.f(lv, B * Z, "lv");
  float* pe = o.f(eps, B * Z, "eps");
  float* pdz = o.f(dz, B * Z, "dz");
  float* pa = o.f(act, B, "act");
  float* pdm = o.f(dmu, B * Z, "dmu");
  float* pdl = o.f(dlv, B * Z, "dlv");
  void* pdmb = o.need(dmu_bf16, BF16, mat(B, Z, ld_b), "dmu_bf16");
  void* pdlb = o.need(dlv_bf16, BF16, mat(B, Z, ld_b), "dlv_bf16");
  GUARD(o);
  check(mog_vae_sample_backward(B, Z, v_pm, v_pv, grad_scale, pm, pl, pe, pdz, pa, pdm, pdl, pdmb,
                                pdlb, ld_b, o.stream()),
        o.name);
}

void sigmoid_backward_(const Tensor& r, const Tensor& dr, Tensor dm, int64_t n) {
  Op o("sigmoid_backward_");
  const bool bf = dm.scalar_type() == BF16;
  void* pdm = o.need(dm, bf ? BF16 : F32, n, "dm");
  float* pr = o.f(r, n, "r");
  float* pdr = o.f(dr, n, "dr");
  GUARD(o);
  check(mog_sigmoid_backward(pr, pdr, pdm, n, bf, o.stream()), o.name);
}

void stn_vae_step_(int64_t B, int64_t C, const Tensor& x, const Tensor& theta_f,
                   const Tensor& theta_b, const Tensor& mask, const Tensor& zval,
                   const Tensor& eps_z, const optional<Tensor>& eps_x, int64_t eps_seed,
                   int64_t eps_offset, bool eps_gen, at::TensorList wt, at::TensorList bias,
                   double lik_std, double v_pm, double v_pv, double v_plv, Tensor canvas_part,
                   Tensor part_rows, const optional<Tensor>& runloss, Tensor vkl,
                   const optional<Tensor>& gb, const optional<Tensor>& a1b,
                   const optional<Tensor>& a2b, const optional<Tensor>& mu,
                   const optional<Tensor>& lv, const optional<Tensor>& z,
                   const optional<Tensor>& zb, const optional<Tensor>& d1b,
                   const optional<Tensor>& d2b, Tensor r, int64_t x_period) {
  Op o("stn_vae_step_");
  TORCH_CHECK(wt.size() == 7 && bias.size() == 7, o.name, ": 7 VAE layers");
  const int64_t C2 = C * C;
  float* pr = o.f(r, B * 784, "r");
  // bf16 W^T packs in MFMA B-fragment order: [out padded to 16][in padded to 32]
  static const int64_t pack[7] = {512 * 800, 256 * 512, 64 * 256, 64 * 256, 256 * 64, 512 * 256,
                                  784 * 512};
  static const int64_t nb[7] = {512, 256, 50, 50, 256, 512, 784};
  vector<void*> w, b;
  for (int k = 0; k < 7; ++k) {
    w.push_back(o.need(wt[k], BF16, pack[k], "wt"));
    b.push_back(o.need(bias[k], F32, nb[k], "bias"));
  }
  float* px = o.f(x, (x_period > 0 ? x_period : B) * C2, "x");
  float* ptf = o.f(theta_f, 6 * B, "theta_f");
  float* ptb = o.f(theta_b, 6 * B, "theta_b");
  float* pm = o.f(mask, B, "mask");
  float* pzv = o.f(zval, B, "zval");
  float* pez = o.f(eps_z, 50 * B, "eps_z");
  float* pex = o.f(eps_x, 784 * B, "eps_x");
  float* pcp = o.f(canvas_part, B * C2, "canvas_part");
  int* prw = o.i(part_rows, B, "part_rows");
  float* prl = o.f(runloss, B, "runloss");
  float* pk = o.f(vkl, B, "vkl");
  void* pgb = o.need(gb, BF16, B * 784, "gb");
  void* pa1 = o.need(a1b, BF16, B * 512, "a1b");
  void* pa2 = o.need(a2b, BF16, B * 256, "a2b");
  float* pmu = o.f(mu, B * 50, "mu");
  float* plv = o.f(lv, B * 50, "lv");
  float* pz = o.f(z, B * 50, "z");
  void* pzb = o.need(zb, BF16, B * 56, "zb");
  void* pd1 = o.need(d1b, BF16, B * 256, "d1b");
  void* pd2 = o.need(d2b, BF16, B * 512, "d2b");
  GUARD(o);
  check(mog_stn_vae_step_forward(B, C, 28, 512, 256, 50, 256, 512, px, ptf, ptb, pm, pzv, pez,
                                 pex, eps_gen, (unsigned long long)eps_seed,
                                 (unsigned long long)eps_offset, arr<void>(w), arr<float>(b),
                                 lik_std, v_pm, v_pv, v_plv, pcp, prw, prl, pk, pgb, pa1, pa2, pmu,
                                 plv, pz, pzb, pd1, pd2, pr, x_period, o.stream()),
        o.name);
}

void pack_frag_f32_(at::TensorList W, at::IntArrayRef K, at::IntArrayRef N,
                    const c10::List<optional<Tensor>>& out) {
  Op o("pack_frag_f32_");
  const int n = (int)W.size();
  TORCH_CHECK(n >= 1 && n <= 8 && (int)K.size() == n && (int)N.size() == n && (int)out.size() == n,
              o.name, ": 1..8 matrices with K, N and an output each");
  vector<void*> w, d;
  vector<int> k, nn;
  for (int i = 0; i < n; ++i) {
    TORCH_CHECK(K[i] > 0 && N[i] > 0, o.name, ": K, N > 0");
    w.push_back(o.f(W[i], K[i] * N[i], "W"));
    const optional<Tensor> oi = out.get(i);
    TORCH_CHECK(oi.has_value(), o.name, ": out given");
    d.push_back(o.f(oi, (K[i] + 15) / 16 * ((N[i] + 15) / 16) * 256, "out"));
    k.push_back((int)K[i]);
    nn.push_back((int)N[i]);
  }
  GUARD(o);
  check(mog_pack_frag_f32(n, arr<float>(w), k.data(), nn.data(), marr<float>(d), o.stream()),
        o.name);
}

void stn_vae_step_f32_(int64_t B, int64_t C, const Tensor& x, const Tensor& theta_f,
                       const Tensor& theta_b, const Tensor& mask, const Tensor& zval,
                       const Tensor& eps_z, const optional<Tensor>& eps_x, int64_t eps_seed,
                       int64_t eps_offset, bool eps_gen, at::TensorList wt, at::TensorList bias,
                       double lik_std, double v_pm, double v_pv, double v_plv,
                       Tensor canvas_part, Tensor part_rows, const optional<Tensor>& runloss,
                       Tensor vkl, const c10::List<optional<Tensor>>& saved, Tensor z, Tensor r,
                       int64_t x_period) {
  Op o("stn_vae_step_f32_");
  TORCH_CHECK(wt.size() == 7 && bias.size() == 7, o.name, ": 7 VAE layers");
  TORCH_CHECK(saved.size() == 11, o.name,
              ": saved = [g, a1pre, a1, a2pre, a2, mu, lv, d1pre, d1, d2pre, d2]");
  const int64_t C2 = C * C;
  // fp32 B-fragment packs: (K + 15) / 16 x (N + 15) / 16 KiB
  static const int64_t pack[7] = {49 * 32 * 256, 32 * 16 * 256, 16 * 4 * 256, 16 * 4 * 256,
                                  4 * 16 * 256, 16 * 32 * 256, 32 * 49 * 256};
  static const int64_t nb[7] = {512, 256, 50, 50, 256, 512, 784};
  vector<void*> w, b;
  for (int k = 0; k < 7; ++k) {
    w.push_back(o.f(wt[k], pack[k], "wt"));
    b.push_back(o.f(bias[k], nb[k], "bias"));
  }
  static const int64_t cols[11] = {784, 512, 512, 256, 256, 50, 50, 256, 256, 512, 512};
  static const char* names[11] = {"g", "a1pre", "a1", "a2pre", "a2", "mu", "lv",
                                  "d1pre", "d1", "d2pre", "d2"};
  vector<void*> sv;
  for (int k = 0; k < 11; ++k) sv.push_back(o.f(saved.get(k), B * cols[k], names[k]));
  float* px = o.f(x, (x_period > 0 ? x_period : B) * C2, "x");
  float* ptf = o.f(theta_f, 6 * B, "theta_f");
  float* ptb = o.f(theta_b, 6 * B, "theta_b");
  float* pm = o.f(mask, B, "mask");
  float* pzv = o.f(zval, B, "zval");
  float* pez = o.f(eps_z, 50 * B, "eps_z");
  float* pex = o.f(eps_x, 784 * B, "eps_x");
  float* pcp = o.f(canvas_part, B * C2, "canvas_part");
  int* prw = o.i(part_rows, B, "part_rows");
  float* prl = o.f(runloss, B, "runloss");
  float* pk = o.f(vkl, B, "vkl");
  float* pz = o.f(z, B * 50, "z");
  float* pr = o.f(r, B * 784, "r");
  auto S = [&](int k) { return reinterpret_cast<float*>(sv[k]); };
  GUARD(o);
  check(mog_stn_vae_step_forward_f32(B, C, px, ptf, ptb, pm, pzv, pez, pex, eps_gen,
                                     (unsigned long long)eps_seed, (unsigned long long)eps_offset,
                                     arr<float>(w), arr<float>(b), lik_std, v_pm, v_pv, v_plv, pcp,
                                     prw, prl, pk, S(0), S(1), S(2), S(3), S(4), S(5), S(6), pz,
                                     S(7), S(8), S(9), S(10), pr, x_period, o.stream()),
        o.name);
}

// ------------------------------------------------- loss / optimizer / RNG ----
void recon_loss_(const Tensor& x, const optional<Tensor>& canvas, const optional<Tensor>& parts,
                 int64_t nparts, int64_t part_stride, const optional<Tensor>& part_rows, int64_t C,
                 const Tensor& runloss, const Tensor& digits, const optional<Tensor>& targets,
                 int64_t B, int64_t C2, double grad_scale, const optional<Tensor>& recon,
                 Tensor bce, Tensor mse, Tensor loss, const optional<Tensor>& acc,
                 const optional<Tensor>& dcanvas) {
  Op o("recon_loss_");
  float* pl = o.f(loss, B, "loss");
  float* px = o.f(x, B * C2, "x");
  float* pc = o.f(canvas, B * C2, "canvas");
  float* pp = o.f(parts, nparts > 0 ? (nparts - 1) * part_stride + B * C2 : 0, "parts");
  const int* prw = o.i(part_rows, nparts * B, "part_rows");
  float* prl = o.f(runloss, B, "runloss");
  const int* pd = o.i(digits, B, "digits");
  const int* pt = o.i(targets, B, "targets");
  float* prc = o.f(recon, B * C2, "recon");
  float* pb = o.f(bce, B, "bce");
  float* pms = o.f(mse, B, "mse");
  float* pa = o.f(acc, B, "acc");
  float* pdc = o.f(dcanvas, B * C2, "dcanvas");
  GUARD(o);
  check(mog_recon_loss(px, pc, pp, nparts, part_stride, prw, C, prl, pd, pt, B, C2, grad_scale,
                       prc, pb, pms, pl, pa, pdc, o.stream()),
        o.name);
}

void batch_mean_(const optional<Tensor>& a0, const optional<Tensor>& a1,
                 const optional<Tensor>& a2, const optional<Tensor>& a3, int64_t B, Tensor out) {
  Op o("batch_mean_");
  float* po = o.f(out, 4, "out");
  float* p0 = o.f(a0, B, "a0");
  float* p1 = o.f(a1, B, "a1");
  float* p2 = o.f(a2, B, "a2");
  float* p3 = o.f(a3, B, "a3");
  GUARD(o);
  check(mog_batch_mean(p0, p1, p2, p3, B, po, o.stream()), o.name);
}

void clip_adam_(Tensor params, Tensor grads, Tensor m, Tensor v, const Tensor& off,
                const Tensor& len, const Tensor& block_tensor, const Tensor& block_start,
                int64_t nblocks, const optional<Tensor>& sumsq, double clip, double lr_t,
                double beta1, double beta2, double eps) {
  // the tensor table lives on the device (off / len / block arrays); the flat
  // buffers must hold the same number of elements
  Op o("clip_adam_");
  const int64_t n = params.numel();
  float* pp = o.f(params, n, "params");
  float* pg = o.f(grads, n, "grads");
  float* pm = o.f(m, n, "m");
  float* pv = o.f(v, n, "v");
  TORCH_CHECK(grads.numel() == n && m.numel() == n && v.numel() == n, o.name,
              ": params / grads / m / v differ in size");
  auto* poff = static_cast<const long*>(o.need(off, at::kLong, 0, "off"));
  auto* plen = static_cast<const long*>(o.need(len, at::kLong, 0, "len"));
  const int* pbt = o.i(block_tensor, nblocks, "block_tensor");
  auto* pbs = static_cast<const long*>(o.need(block_start, at::kLong, nblocks, "block_start"));
  float* ps = o.f(sumsq, nblocks, "sumsq");  // per-chunk scratch
  GUARD(o);
  check(mog_clip_adam(pp, pg, pm, pv, poff, plen, pbt, pbs, nblocks, ps, clip, lr_t, beta1, beta2,
                      eps, o.stream()),
        o.name);
}

void add_(const Tensor& a, const Tensor& b, Tensor out, int64_t n) {
  Op o("add_");
  float* po = o.f(out, n, "out");
  float* pa = o.f(a, n, "a");
  float* pb = o.f(b, n, "b");
  GUARD(o);
  check(mog_add(pa, pb, po, n, o.stream()), o.name);
}

void rng_fill_(Tensor out, int64_t seed, int64_t offset, bool normal) {
  Op o("rng_fill_");
  float* po = o.f(out, out.numel(), "out");
  GUARD(o);
  check(mog_rng_fill(po, out.numel(), (unsigned long long)seed, (unsigned long long)offset, normal,
                     o.stream()),
        o.name);
}

// several noise buffers / 32-bit fills in one launch
void rng_fill_batch_(at::TensorList out, int64_t seed, at::IntArrayRef offset,
                     at::IntArrayRef normal) {
  Op o("rng_fill_batch_");
  TORCH_CHECK(out.size() == offset.size() && out.size() == normal.size(), o.name, ": lengths");
  vector<float*> p;
  vector<long> n;
  vector<unsigned long long> off;
  vector<int> nm;
  for (size_t j = 0; j < out.size(); ++j) {
    p.push_back(o.f(out[j], out[j].numel(), "out"));
    n.push_back(out[j].numel());
    off.push_back((unsigned long long)offset[j]);
    nm.push_back(normal[j] != 0);
  }
  GUARD(o);
  check(mog_rng_fill_batch((int)p.size(), p.data(), n.data(), (unsigned long long)seed, off.data(),
                           nm.data(), o.stream()),
        o.name);
}

// up to 8 same-size 32-bit copies in one launch (mog_copy32_batch)
void copy32_batch_(at::TensorList dst, at::TensorList src) {
  Op o("copy32_batch_");
  TORCH_CHECK(dst.size() == src.size() && dst.size() <= 8, o.name, ": up to 8 dst / src pairs");
  vector<void*> d, a;
  vector<long> n;
  for (size_t j = 0; j < dst.size(); ++j) {
    TORCH_CHECK(dst[j].element_size() == 4 && src[j].element_size() == 4 &&
                    dst[j].numel() == src[j].numel() && dst[j].is_contiguous() &&
                    src[j].is_contiguous(),
                o.name, ": contiguous 32-bit tensors of one size per pair");
    d.push_back(o.need(dst[j], dst[j].scalar_type(), dst[j].numel(), "dst"));
    a.push_back(o.need(src[j], src[j].scalar_type(), src[j].numel(), "src"));
    n.push_back((long)dst[j].numel());
  }
  GUARD(o);
  check(mog_copy32_batch((int)d.size(), d.data(), const_cast<const void* const*>(a.data()),
                         n.data(), o.stream()),
        o.name);
}

// fp32 transposes in one launch (mog_transpose32_batch)
void transpose32_batch_(at::TensorList dst, at::TensorList src) {
  Op o("transpose32_batch_");
  TORCH_CHECK(dst.size() == src.size() && dst.size() <= 8, o.name, ": up to 8 pairs");
  vector<void*> d, a;
  vector<int> r, c;
  for (size_t j = 0; j < dst.size(); ++j) {
    TORCH_CHECK(src[j].dim() == 2 && dst[j].dim() == 2 && src[j].is_contiguous() &&
                    dst[j].is_contiguous() && dst[j].size(0) == src[j].size(1) &&
                    dst[j].size(1) == src[j].size(0),
                o.name, ": contiguous 2-d src [r][c] and dst [c][r]");
    d.push_back(o.f(dst[j], dst[j].numel(), "dst"));
    a.push_back(o.f(src[j], src[j].numel(), "src"));
    r.push_back((int)src[j].size(0));
    c.push_back((int)src[j].size(1));
  }
  GUARD(o);
  check(mog_transpose32_batch((int)d.size(), marr<float>(d), arr<float>(a), r.data(), c.data(),
                              o.stream()),
        o.name);
}

void fill32_batch_(at::TensorList dst, at::IntArrayRef value) {
  Op o("fill32_batch_");
  TORCH_CHECK(dst.size() == value.size(), o.name, ": lengths");
  vector<void*> p;
  vector<long> n;
  vector<unsigned> v;
  for (size_t j = 0; j < dst.size(); ++j) {
    TORCH_CHECK(dst[j].element_size() == 4 && dst[j].is_contiguous(), o.name, ": 32-bit contiguous");
    p.push_back(o.need(dst[j], dst[j].scalar_type(), dst[j].numel(), "dst"));
    n.push_back(dst[j].numel());
    v.push_back((unsigned)value[j]);
  }
  GUARD(o);
  check(mog_fill32_batch((int)p.size(), p.data(), n.data(), v.data(), o.stream()), o.name);
}

void copy_f4_(const Tensor& src, Tensor dst) {
  Op o("copy_f4_");
  TORCH_CHECK(src.numel() == dst.numel() && src.numel() % 4 == 0, "copy_f4_: sizes");
  const float* ps = o.f(src, src.numel(), "src");
  float* pd = o.f(dst, dst.numel(), "dst");
  GUARD(o);
  check(mog_copy_f4(ps, pd, src.numel() / 4, o.stream()), o.name);
}

// ---------------------------------------------- AIR-ASR cells and losses ----
// (air/air_number_bbox_location.py; records [T][28][B], asr_cell.hip)
constexpr int64_t ASR_NQ = 28, ASR_DN = 12;

void asr_pack_(int64_t B, int64_t Z, int64_t H, int64_t ld, const optional<Tensor>& z,
               const optional<Tensor>& ss, const optional<Tensor>& h, Tensor out,
               const optional<Tensor>& h2, const optional<Tensor>& out2) {
  Op o("asr_pack_");
  float* po = o.f(out, B * ld, "out");
  float* pz = o.f(z, B * Z, "z");
  float* ps = o.f(ss, B * 3, "ss");
  float* ph = o.f(h, B * H, "h");
  float* ph2 = o.f(h2, B * H, "h2");
  float* po2 = o.f(out2, B * ld, "out2");
  GUARD(o);
  check(mog_asr_pack(B, Z, H, ld, pz, ps, ph, po, ph2, po2, o.stream()), o.name);
}

void asr_unpack_(int64_t B, int64_t Z, int64_t H, int64_t ld, const Tensor& dU, const Tensor& dUg,
                 Tensor dz, Tensor dss, Tensor dh, Tensor dhg, int64_t acc_dz) {
  Op o("asr_unpack_");
  float* pdz = o.f(dz, B * Z, "dz");
  float* pds = o.f(dss, B * 3, "dss");
  float* pdh = o.f(dh, B * H, "dh");
  float* pdg = o.f(dhg, B * H, "dhg");
  float* pu = o.f(dU, B * ld, "dU");
  float* pug = o.f(dUg, B * ld, "dUg");
  GUARD(o);
  check(mog_asr_unpack(B, Z, H, ld, pu, pug, pdz, pds, pdh, pdg, (int)acc_dz, o.stream()),
        o.name);
}

void asr_unpack_parts_(int64_t B, int64_t Z, int64_t H, int64_t ld, const Tensor& dU,
                       const Tensor& dUg, int64_t nparts, Tensor dz, Tensor dss, Tensor dh,
                       Tensor dhg, int64_t acc_dz) {
  Op o("asr_unpack_parts_");
  float* pdz = o.f(dz, B * Z, "dz");
  float* pds = o.f(dss, B * 3, "dss");
  float* pdh = o.f(dh, B * H, "dh");
  float* pdg = o.f(dhg, B * H, "dhg");
  float* pu = o.f(dU, nparts * B * ld, "dU");
  float* pug = o.f(dUg, nparts * B * ld, "dUg");
  GUARD(o);
  check(mog_asr_unpack_parts(B, Z, H, ld, pu, pug, (int)nparts, B * ld, pdz, pds, pdh, pdg,
                             (int)acc_dz, o.stream()),
        o.name);
}

void asr_step_forward_(int64_t B, int64_t step, bool train, int64_t fix_steps, double thr,
                       double temperature, double s_pm, double s_pv, double s_plv,
                       double gamma_num, at::TensorList w, const c10::List<optional<Tensor>>& hid,
                       const Tensor& eps_shift, const Tensor& eps_scale, const Tensor& u,
                       Tensor stop, Tensor digits, Tensor live, Tensor rec, Tensor theta_fwd,
                       Tensor theta_back, Tensor ss, Tensor scale, Tensor shift, Tensor zprob,
                       Tensor zmask, Tensor zval, Tensor zc) {
  Op o("asr_step_forward_");
  TORCH_CHECK(w.size() == 20 && hid.size() == 8, o.name, ": 10 output layers, 8 hidden layers");
  float* pst = o.f(stop, B, "stop");
  auto pw = o.list(w, F32, 1, "w");
  auto ph = o.list(hid, F32, B * 64, "hid");
  float* peh = o.f(eps_shift, 2 * B, "eps_shift");
  float* pes = o.f(eps_scale, B, "eps_scale");
  float* pu = o.f(u, B, "u");
  int* pd = o.i(digits, B, "digits");
  int* pl = o.i(live, step + 2, "live");
  float* pr = o.f(rec, ASR_NQ * B, "rec");
  float* ptf = o.f(theta_fwd, 6 * B, "theta_fwd");
  float* ptb = o.f(theta_back, 6 * B, "theta_back");
  float* pss = o.f(ss, 3 * B, "ss");
  float* psc = o.f(scale, B, "scale");
  float* psh = o.f(shift, 2 * B, "shift");
  float* pzp = o.f(zprob, B, "zprob");
  float* pzm = o.f(zmask, B, "zmask");
  float* pzv = o.f(zval, B, "zval");
  float* pzc = o.f(zc, B, "zc");
  GUARD(o);
  check(mog_asr_step_forward(B, step, train, fix_steps, thr, temperature, s_pm, s_pv, s_plv,
                             gamma_num, arr<float>(pw), marr<float>(ph), peh, pes, pu, pst, pd, pl,
                             pr, ptf, ptb, pss, psc, psh, pzp, pzm, pzv, pzc, o.stream()),
        o.name);
}

void asr_terms_(int64_t B, int64_t T, int64_t C, at::IntArrayRef cons, at::ArrayRef<double> gammas,
                const Tensor& rec, const Tensor& vkl, const Tensor& zmask, const Tensor& live,
                Tensor klsum, Tensor pr, Tensor area, Tensor out, Tensor size, Tensor overlap,
                Tensor zsum) {
  Op o("asr_terms_");
  TORCH_CHECK(gammas.size() == 8 && !cons.empty() && cons.size() <= 8, o.name,
              ": 8 gammas, 1..8 counts");
  vector<int> c(cons.begin(), cons.end());
  vector<float> g(gammas.begin(), gammas.end());
  float* pk = o.f(klsum, B, "klsum");
  float* pp = o.f(pr, B, "pr");
  float* pa = o.f(area, B, "area");
  float* pout = o.f(out, B, "out");
  float* psz = o.f(size, B, "size");
  float* pov = o.f(overlap, B, "overlap");
  float* pzs = o.f(zsum, T, "zsum");
  float* prec = o.f(rec, T * ASR_NQ * B, "rec");
  float* pv = o.f(vkl, T * B, "vkl");
  float* pzm = o.f(zmask, T * B, "zmask");
  const int* pl = o.i(live, T + 1, "live");
  GUARD(o);
  check(mog_asr_terms(B, T, C, (int)c.size(), c.data(), g.data(), prec, pv, pzm, pl, pk, pp, pa,
                      pout, psz, pov, pzs, o.stream()),
        o.name);
}

void asr_finalize_(int64_t B, int64_t T, int64_t C, at::IntArrayRef cons,
                   at::ArrayRef<double> gammas, double inv_batch_global, const Tensor& rec,
                   const Tensor& live, const Tensor& zsum, const Tensor& pr, Tensor loss,
                   Tensor element, Tensor margin) {
  Op o("asr_finalize_");
  TORCH_CHECK(gammas.size() == 8 && !cons.empty() && cons.size() <= 8, o.name,
              ": 8 gammas, 1..8 counts");
  vector<int> c(cons.begin(), cons.end());
  vector<float> g(gammas.begin(), gammas.end());
  float* pl = o.f(loss, B, "loss");
  float* pe = o.f(element, B, "element");
  float* pm = o.f(margin, 1, "margin");
  float* prec = o.f(rec, T * ASR_NQ * B, "rec");
  const int* plv = o.i(live, T + 1, "live");
  float* pzs = o.f(zsum, T, "zsum");
  float* pp = o.f(pr, B, "pr");
  GUARD(o);
  check(mog_asr_finalize(B, T, C, (int)c.size(), c.data(), g.data(), inv_batch_global, prec, plv,
                         pzs, pp, pl, pe, pm, o.stream()),
        o.name);
}

void asr_terms_backward_(int64_t B, int64_t T, int64_t C, at::IntArrayRef cons,
                         at::ArrayRef<double> gammas, double grad_scale, double inv_batch_global,
                         const Tensor& rec, const Tensor& live, const Tensor& zsum, Tensor dreg) {
  Op o("asr_terms_backward_");
  TORCH_CHECK(gammas.size() == 8 && !cons.empty() && cons.size() <= 8, o.name,
              ": 8 gammas, 1..8 counts");
  vector<int> c(cons.begin(), cons.end());
  vector<float> g(gammas.begin(), gammas.end());
  float* pd = o.f(dreg, T * 4 * B, "dreg");
  float* prec = o.f(rec, T * ASR_NQ * B, "rec");
  const int* pl = o.i(live, T + 1, "live");
  float* pzs = o.f(zsum, T, "zsum");
  GUARD(o);
  check(mog_asr_terms_backward(B, T, C, (int)c.size(), c.data(), g.data(), grad_scale,
                               inv_batch_global, prec, pl, pzs, pd, o.stream()),
        o.name);
}

void asr_step_backward_(int64_t B, bool train, int64_t fix_steps, double temperature,
                        double s_pm, double s_pv, double grad_scale, at::TensorList w,
                        const c10::List<optional<Tensor>>& hid, const Tensor& rec,
                        const Tensor& eps_shift, const Tensor& eps_scale,
                        const Tensor& dtheta_fwd, const Tensor& dtheta_back, const Tensor& dot,
                        const Tensor& dreg, const optional<Tensor>& dss, Tensor douts,
                        const c10::List<optional<Tensor>>& dpre) {
  Op o("asr_step_backward_");
  TORCH_CHECK(w.size() == 20 && hid.size() == 8 && dpre.size() == 8, o.name,
              ": 10 output layers, 8 hidden layers");
  float* pdo = o.f(douts, B * ASR_DN, "douts");
  auto pw = o.list(w, F32, 1, "w");
  auto ph = o.list(hid, F32, B * 64, "hid");
  auto pdp = o.list(dpre, F32, B * 64, "dpre");
  float* prec = o.f(rec, ASR_NQ * B, "rec");
  float* peh = o.f(eps_shift, 2 * B, "eps_shift");
  float* pes = o.f(eps_scale, B, "eps_scale");
  float* ptf = o.f(dtheta_fwd, 6 * B, "dtheta_fwd");
  float* ptb = o.f(dtheta_back, 6 * B, "dtheta_back");
  float* pd = o.f(dot, B, "dot");
  float* pdr = o.f(dreg, 4 * B, "dreg");
  float* pds = o.f(dss, 3 * B, "dss");
  GUARD(o);
  check(mog_asr_step_backward(B, train, fix_steps, temperature, s_pm, s_pv, grad_scale,
                              arr<float>(pw), marr<float>(ph), prec, peh, pes, ptf, ptb, pd, pdr,
                              pds, pdo, marr<float>(pdp), o.stream()),
        o.name);
}

}  // namespace

// split-K partials of the TN forms: reduce = 1 -> a transient [splitk][M][N]
// (+ [splitk][N] column-sum partials) fp32 workspace from the caching
// allocator (on the op's stream) summed into C and the column sums in a fixed
// order after the GEMM (deterministic); 0 -> float atomics into C
Tensor splitk_work(const Op& o, int64_t splitk, int64_t M, int64_t N, int64_t reduce) {
  if (!reduce || splitk <= 1 || M <= 0 || N <= 0) return Tensor();
  return at::empty({splitk * (M * N + N)}, at::TensorOptions().dtype(F32).device(*o.dev));
}

void gemm_f32_x3_tn_(const Tensor& A, const Tensor& B, Tensor C, const optional<Tensor>& colsum,
                     int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                     int64_t splitk, int64_t reduce) {
  Op o("gemm_f32_x3_tn_");
  float* c = o.f(C, mat(M, N, ldc), "C");
  float* a = o.f(A, mat(K, M, lda), "A");
  float* b = o.f(B, mat(K, N, ldb), "B");
  float* cs = o.f(colsum, N, "colsum");
  GUARD(o);
  Tensor w = splitk_work(o, splitk, M, N, reduce);
  check(mog_gemm_f32_x3_tn(a, b, c, cs, M, N, K, lda, ldb, ldc, splitk,
                           w.defined() ? w.data_ptr<float>() : nullptr,
                           w.defined() ? w.numel() : 0, o.stream()),
        o.name);
}

void split3_bf16_(const Tensor& src, Tensor dst, int64_t rows, int64_t cols, int64_t ld_src,
                  int64_t ld_dst, int64_t piece_stride) {
  Op o("split3_bf16_");
  const float* a = o.f(src, mat(rows, cols, ld_src), "src");
  void* d = o.need(dst, BF16, 2 * piece_stride + mat(rows, ld_dst, ld_dst), "dst");
  GUARD(o);
  check(mog_split3_bf16(a, rows, cols, ld_src, d, ld_dst, piece_stride, o.stream()), o.name);
}

void split3_sum_bf16_(const Tensor& src, int64_t nsum, int64_t sum_stride, Tensor dst,
                      int64_t rows, int64_t cols, int64_t ld_src, int64_t ld_dst,
                      int64_t piece_stride) {
  Op o("split3_sum_bf16_");
  const float* a = o.f(src, (nsum - 1) * sum_stride + mat(rows, cols, ld_src), "src");
  void* d = o.need(dst, BF16, 2 * piece_stride + mat(rows, ld_dst, ld_dst), "dst");
  GUARD(o);
  check(mog_split3_sum_bf16(a, nsum, sum_stride, rows, cols, ld_src, d, ld_dst, piece_stride,
                            o.stream()),
        o.name);
}

void gemm_x3p_tn_(const Tensor& A3, int64_t sa, const Tensor& B3, int64_t sb, Tensor C,
                  const optional<Tensor>& colsum, int64_t M, int64_t N, int64_t K, int64_t lda,
                  int64_t ldb, int64_t ldc, int64_t splitk, int64_t npieces, int64_t reduce) {
  Op o("gemm_x3p_tn_");
  float* c = o.f(C, mat(M, N, ldc), "C");
  const int64_t np1 = npieces - 1;
  // the kernel reads 16-byte chunks (8 bf16) of every k-row: the last row of
  // the last piece is read up to round8(M) / round8(N) elements
  auto ext = [](int64_t K, int64_t n, int64_t ld) { return K > 0 ? (K - 1) * ld + (n + 7) / 8 * 8 : 0; };
  const void* a = o.need(A3, BF16, np1 * sa + ext(K, M, lda), "A3");
  const void* b = o.need(B3, BF16, np1 * sb + ext(K, N, ldb), "B3");
  float* cs = o.f(colsum, N, "colsum");
  GUARD(o);
  Tensor w = splitk_work(o, splitk, M, N, reduce);
  check(mog_gemm_x3p_tn(a, sa, b, sb, c, cs, M, N, K, lda, ldb, ldc, splitk, npieces,
                        w.defined() ? w.data_ptr<float>() : nullptr, w.defined() ? w.numel() : 0,
                        o.stream()),
        o.name);
}

// the grouped tall-K bf16 weight gradients (wgrad_tn.hip): out[i] += X[i]^T
// dY[i] over K rows, colsum[i] += column sums of dY[i]; dims holds (M, N,
// lda, ldb, ldc) per problem.  The kernel reads whole k-rows of both operands
// (K x ld elements each); the [nsplit][tiles] partial workspace is a transient
// of the caching allocator on the op's stream.
void wgrad_tn_(at::TensorList X, at::TensorList dY, at::TensorList out,
               const c10::List<optional<Tensor>>& colsum, at::IntArrayRef dims, int64_t K,
               int64_t nsplit, bool x3) {
  Op o(x3 ? "wgrad_tn_x3_" : "wgrad_tn_bf16_");
  const size_t n = out.size();
  TORCH_CHECK(n >= 1 && n <= 8 && X.size() == n && dY.size() == n && colsum.size() == n &&
                  dims.size() == 5 * n,
              o.name, ": 1-8 problems, X / dY / out / colsum of one length n, 5 n dims");
  vector<void*> xs, ys, os, cs;
  vector<int> d;
  for (size_t i = 0; i < n; ++i) {
    const int64_t M = dims[5 * i], N = dims[5 * i + 1], lda = dims[5 * i + 2],
                  ldb = dims[5 * i + 3], ldc = dims[5 * i + 4];
    TORCH_CHECK(M > 0 && N > 0 && lda >= M && ldb >= N && ldc >= N, o.name,
                ": bad dims of problem ", i);
    os.push_back(o.f(out[i], mat(M, N, ldc), "out"));
    xs.push_back(o.need(X[i], x3 ? F32 : BF16, K * lda, "X"));
    ys.push_back(o.need(dY[i], x3 ? F32 : BF16, K * ldb, "dY"));
    cs.push_back(o.f(static_cast<optional<Tensor>>(colsum[i]), N, "colsum"));
    for (int64_t v : {M, N, lda, ldb, ldc}) d.push_back((int)v);
  }
  GUARD(o);
  const long we = mog_wgrad_tn_work_elems((int)n, d.data(), (int)nsplit);
  TORCH_CHECK(we > 0, o.name, ": bad problem set");
  Tensor w = at::empty({we}, at::TensorOptions().dtype(F32).device(*o.dev));
  const int rc = x3 ? mog_wgrad_tn_x3((int)n, arr<float>(xs), arr<float>(ys), marr<float>(os),
                                      marr<float>(cs), d.data(), (int)K, (int)nsplit,
                                      w.data_ptr<float>(), we, o.stream())
                   : mog_wgrad_tn_bf16((int)n, arr<void>(xs), arr<void>(ys), marr<float>(os),
                                       marr<float>(cs), d.data(), (int)K, (int)nsplit,
                                       w.data_ptr<float>(), we, o.stream());
  check(rc, o.name);
}

// the heads' output-layer weight / bias gradients (mog_heads_output_wgrad),
// the chunk-partial workspace a transient of the caching allocator
void heads_output_wgrad_(at::TensorList hid, at::TensorList dout, at::TensorList gw,
                         const c10::List<optional<Tensor>>& gb, at::IntArrayRef k, int64_t R,
                         int64_t HS) {
  Op o("heads_output_wgrad_");
  const size_t n = hid.size();
  TORCH_CHECK(n >= 1 && n <= 5 && dout.size() == n && gw.size() == n && gb.size() == n &&
                  k.size() == n,
              o.name, ": 1-5 heads, one hid / dout / gw / gb / k each");
  vector<int> kk;
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(k[i] == 1 || k[i] == 2, o.name, ": k is 1 or 2");
    kk.push_back((int)k[i]);
  }
  auto gws = [&] {
    vector<void*> v;
    for (size_t i = 0; i < n; ++i) v.push_back(o.f(gw[i], HS * k[i], "gw"));
    return v;
  }();
  auto h = o.list(hid, F32, R * HS, "hid"), d = o.list(dout, F32, R * 2, "dout");
  vector<void*> b;
  for (size_t i = 0; i < n; ++i) b.push_back(o.f(static_cast<optional<Tensor>>(gb[i]), k[i], "gb"));
  GUARD(o);
  const long we = mog_heads_output_wgrad_work_elems((int)n, (int)R, (int)HS);
  TORCH_CHECK(we > 0, o.name, ": bad shape");
  Tensor w = at::empty({we}, at::TensorOptions().dtype(F32).device(*o.dev));
  check(mog_heads_output_wgrad((int)n, arr<float>(h), arr<float>(d), marr<float>(gws),
                               marr<float>(b), kk.data(), (int)R, (int)HS, w.data_ptr<float>(),
                               we, o.stream()),
        o.name);
}

void wgrad_tn_bf16_(at::TensorList X, at::TensorList dY, at::TensorList out,
                    const c10::List<optional<Tensor>>& colsum, at::IntArrayRef dims, int64_t K,
                    int64_t nsplit) {
  wgrad_tn_(X, dY, out, colsum, dims, K, nsplit, false);
}

void wgrad_tn_x3_(at::TensorList X, at::TensorList dY, at::TensorList out,
                  const c10::List<optional<Tensor>>& colsum, at::IntArrayRef dims, int64_t K,
                  int64_t nsplit) {
  wgrad_tn_(X, dY, out, colsum, dims, K, nsplit, true);
}

// out[i][M,N] += X[i]^T dY[i] over K rows (+ bias[i] += colsum(dY[i])) for
// every problem i in ONE launch; dims holds (M, N, K, lda, ldb, ldc) per
// problem.  Every operand is checked for the extent its problem touches and
// the written ones are alias-annotated in the schema; the device pointer table
// of the C ABI is built here.
void gemm_f32_wgrad_group_(at::TensorList X, at::TensorList dY, at::TensorList out,
                           const c10::List<optional<Tensor>>& bias, at::IntArrayRef dims) {
  Op o("gemm_f32_wgrad_group_");
  const size_t n = out.size();
  TORCH_CHECK(n > 0 && X.size() == n && dY.size() == n && bias.size() == n && dims.size() == 6 * n,
              o.name, ": X, dY, out, bias of one length n and 6 n dims");
  vector<long long> table;
  table.reserve(10 * n);
  for (size_t i = 0; i < n; ++i) {
    const int64_t M = dims[6 * i], N = dims[6 * i + 1], K = dims[6 * i + 2];
    const int64_t lda = dims[6 * i + 3], ldb = dims[6 * i + 4], ldc = dims[6 * i + 5];
    TORCH_CHECK(M > 0 && N > 0 && K >= 0 && lda >= M && ldb >= N && ldc >= N, o.name,
                ": bad dims of problem ", i);
    void* c = o.f(out[i], mat(M, N, ldc), "out");
    void* a = o.f(X[i], mat(K, M, lda), "X");
    void* b = o.f(dY[i], mat(K, N, ldb), "dY");
    void* bi = o.f(static_cast<optional<Tensor>>(bias[i]), N, "bias");
    for (long long v : {(long long)(uintptr_t)a, (long long)(uintptr_t)b, (long long)(uintptr_t)c,
                        (long long)(uintptr_t)bi, (long long)M, (long long)N, (long long)K,
                        (long long)lda, (long long)ldb, (long long)ldc})
      table.push_back(v);
  }
  GUARD(o);
  check(mog_gemm_f32_wgrad_group(table.data(), (int)n, o.stream()), o.name);
}

void gemm_x3_nt_(const Tensor& A, const Tensor& B3, int64_t sb, Tensor C,
                 const optional<Tensor>& aux, int64_t M, int64_t N, int64_t K, int64_t lda,
                 int64_t ldb, int64_t ldc, int64_t ldaux, int64_t epi) {
  Op o("gemm_x3_nt_");
  float* c = o.f(C, mat(M, N, ldc), "C");
  const float* a = o.f(A, mat(M, K, lda), "A");
  const void* b = o.need(B3, BF16, 2 * sb + mat(N, ldb, ldb), "B3");
  const float* x = o.f(aux, mat(M, N, ldaux), "aux");
  GUARD(o);
  check(mog_gemm_x3_nt(a, b, sb, c, x, M, N, K, lda, ldb, ldc, ldaux, epi, o.stream()), o.name);
}

TORCH_LIBRARY_FRAGMENT(mog_air, m) {
  m.def(
      "gemm_x3_nt_(Tensor A, Tensor B3, int sb, Tensor(a!) C, Tensor? aux, int M, int N, int K, "
      "int lda, int ldb, int ldc, int ldaux, int epi) -> ()");
  m.def(
      "gemm_f32_wgrad_group_(Tensor[] X, Tensor[] dY, Tensor(a!)[] out, Tensor(b!)?[] bias, "
      "int[] dims) -> ()");
  m.def(
      "wgrad_tn_bf16_(Tensor[] X, Tensor[] dY, Tensor(a!)[] out, Tensor(b!)?[] colsum, int[] dims, "
      "int K, int nsplit) -> ()");
  m.def(
      "wgrad_tn_x3_(Tensor[] X, Tensor[] dY, Tensor(a!)[] out, Tensor(b!)?[] colsum, int[] dims, "
      "int K, int nsplit) -> ()");
  m.def(
      "split3_bf16_(Tensor src, Tensor(a!) dst, int rows, int cols, int ld_src, int ld_dst, "
      "int piece_stride) -> ()");
  m.def(
      "gemm_x3p_tn_(Tensor A3, int sa, Tensor B3, int sb, Tensor(a!) C, Tensor(b!)? colsum, "
      "int M, int N, int K, int lda, int ldb, int ldc, int splitk, int npieces=3, int reduce=1) -> ()");
  m.def(
      "gemm_f32_x3_tn_(Tensor A, Tensor B, Tensor(a!) C, Tensor(b!)? colsum, int M, int N, "
      "int K, int lda, int ldb, int ldc, int splitk, int reduce=1) -> ()");
  m.def(
      "gemm_f32_(Tensor[] A, Tensor[] B, Tensor(a!)[] C, Tensor?[] bias, Tensor?[] Cin, "
      "Tensor(b!)?[] Cpre, Tensor?[] aux, Tensor(c!)?[] colsum, int M, int N, int K, int lda, "
      "int ldb, int ldc, int ldaux, bool transA, bool transB, int epi, float aux_scale, "
      "int splitk) -> ()");
  m.def(
      "gemm_f32_sigmoid_philox_(Tensor A, Tensor B, Tensor(a!) C, Tensor? bias, int M, int N, "
      "int K, int lda, int ldb, int ldc, float scale, int seed, int offset) -> ()");
  m.def(
      "gemm_f32_kseg_(Tensor[] A, Tensor[] B, Tensor(a!) C, Tensor? bias, Tensor? Cin, int M, "
      "int N, int kseg, int lda, int ldb, int ldc, bool transA, bool transB, int epi) -> ()");
  m.def(
      "gemm_f32_kseg_group_(Tensor[] A, Tensor[] B, Tensor(a!)[] C, Tensor?[] Cin, int[] nseg, "
      "int M, int N, int kseg, int lda, int ldb, int ldc, bool transB) -> ()");
  m.def(
      "gemm_bf16_(Tensor[] A, Tensor[] B, Tensor(a!)[] C, Tensor?[] bias, Tensor?[] Cin, "
      "Tensor?[] aux, Tensor(b!)?[] colsum, int M, int N, int K, int lda, int ldb, int ldc, "
      "int ldaux, bool tn, int epi, float aux_scale, int splitk) -> ()");
  m.def("cvt_bf16_batch_(Tensor[] src, Tensor(a!)[] dst, int[] dims) -> ()");
  m.def(
      "stn_forward_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, int Wout, "
      "Tensor(a!) out, Tensor? z, Tensor? mask, int mode, int u_period=0) -> ()");
  m.def(
      "stn_backward_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, int Wout, "
      "Tensor G, Tensor? gscale, Tensor(a!)? dU, Tensor(b!)? dtheta, Tensor(c!)? dot, "
      "int u_period, int g_period) -> ()");
  m.def(
      "stn_backward_sigmoid_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, "
      "int Wout, Tensor G, Tensor? gscale, Tensor(a!) dm, Tensor(b!)? dtheta, Tensor(c!)? dot, "
      "int g_period) -> ()");
  m.def(
      "lstm_cell_forward_(Tensor G, Tensor? bias, Tensor? c_prev, Tensor(a!) c_out, "
      "Tensor(b!) h_out, int B, int H) -> ()");
  m.def(
      "lstm_cell_backward_(Tensor G, Tensor? bias, Tensor? c_prev, Tensor c_cur, Tensor dh, "
      "Tensor? dc, Tensor(a!) dG, Tensor(b!) dc_prev, Tensor(c!)? dGsum, int B, int H) -> ()");
  m.def(
      "lstm_cell_forward2_(Tensor G0, Tensor? c_prev0, Tensor(a!) c_out0, Tensor(b!) h_out0, "
      "Tensor G1, Tensor? c_prev1, Tensor(c!) c_out1, Tensor(d!) h_out1, int B, int H) -> ()");
  m.def(
      "lstm_cell_backward2_(Tensor G0, Tensor? c_prev0, Tensor c_cur0, Tensor dh0, Tensor? dc0, "
      "Tensor(a!) dG0, Tensor(b!) dc_prev0, Tensor(c!)? dGsum0, Tensor G1, Tensor? c_prev1, "
      "Tensor c_cur1, Tensor dh1, Tensor? dc1, Tensor(d!) dG1, Tensor(e!) dc_prev1, "
      "Tensor(f!)? dGsum1, int B, int H) -> ()");
  m.def(
      "heads_output_wgrad_(Tensor[] hid, Tensor[] dout, Tensor(a!)[] gw, Tensor(b!)?[] gb, "
      "int[] k, int R, int HS) -> ()");
  m.def(
      "split3_sum_bf16_(Tensor src, int nsum, int sum_stride, Tensor(a!) dst, int rows, "
      "int cols, int ld_src, int ld_dst, int piece_stride) -> ()");
  m.def(
      "lstm_cell_backward_parts_(Tensor G, Tensor? bias, Tensor? c_prev, Tensor c_cur, "
      "Tensor dh, Tensor dh_parts, int nparts, Tensor? dc, Tensor(a!) dG, Tensor(b!) dc_prev, "
      "Tensor(c!)? dGsum, int B, int H) -> ()");
  m.def(
      "asr_unpack_parts_(int B, int Z, int H, int ld, Tensor dU, Tensor dUg, int nparts, "
      "Tensor(a!) dz, Tensor(b!) dss, Tensor(c!) dh, Tensor(d!) dhg, int acc_dz) -> ()");
  m.def("copy32_batch_(Tensor(a!)[] dst, Tensor[] src) -> ()");
  m.def("transpose32_batch_(Tensor(a!)[] dst, Tensor[] src) -> ()");
  m.def(
      "air_step_forward_(int B, int HS, int HZ, int step, bool train, bool use_num_prior, "
      "float thr, float temperature, float prior_lo, float prior_bias, float s_pm, float s_pv, "
      "float s_plv, float h_pm, float h_pv, float h_plv, Tensor[] hid, Tensor[] w2, "
      "Tensor[] b2, Tensor eps_scale, Tensor eps_shift, Tensor u, Tensor(a!) stop, "
      "Tensor(b!) runloss, Tensor(c!) digits, Tensor(d!) live, Tensor(e!) rec, "
      "Tensor(f!) theta_fwd, Tensor(g!) theta_back, Tensor(h!) scale, Tensor(i!) shift, "
      "Tensor(j!) zprob, Tensor(k!) zkl, Tensor(l!) skl, Tensor(m!) shkl, Tensor(n!) zmask, "
      "Tensor(o!) zval, Tensor(p!) zc, Tensor? prior_lo_dev=None) -> ()");
  m.def(
      "air_step_forward_steps_(int steps, int B, int HS, int HZ, bool train, bool use_num_prior, "
      "float thr, float temperature, float prior_lo, float[] prior_bias, float s_pm, float s_pv, "
      "float s_plv, float h_pm, float h_pv, float h_plv, Tensor[] hid, Tensor[] w2, "
      "Tensor[] b2, Tensor eps_scale, Tensor eps_shift, Tensor u, Tensor(a!) stop, "
      "Tensor(c!) digits, Tensor(d!) live, Tensor(e!) rec, "
      "Tensor(f!) theta_fwd, Tensor(g!) theta_back, Tensor(h!) scale, Tensor(i!) shift, "
      "Tensor(j!) zprob, Tensor(k!) zkl, Tensor(l!) skl, Tensor(m!) shkl, Tensor(n!) zmask, "
      "Tensor(o!) zval, Tensor(p!) zc, Tensor? prior_lo_dev=None) -> ()");
  m.def(
      "air_step_backward_(int B, int HS, bool train, bool use_num_prior, float temperature, "
      "float prior_lo, float prior_bias, float s_pm, float s_pv, float h_pm, float h_pv, "
      "float grad_scale, Tensor? dloss, Tensor rec, Tensor eps_scale, Tensor eps_shift, "
      "Tensor dtheta_fwd, Tensor dtheta_back, Tensor dot, Tensor[] hid, Tensor[] w2, "
      "Tensor(a!) dout, int dout_hs, Tensor(b!) dhid, int dhid_hs, Tensor? prior_lo_dev=None, "
      "int steps=1) -> ()");
  m.def(
      "generation_prior_(int G, int Z, float s_pm, float s_plv, float h_pm, float h_plv, "
      "float v_pm, float v_plv, Tensor eps_scale, Tensor eps_shift, Tensor eps_z, "
      "Tensor(a!) theta_back, Tensor(b!) scale, Tensor(c!) shift, Tensor(d!) z) -> ()");
  m.def(
      "stn_write_parts_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, int Wout, "
      "Tensor z, Tensor mask, Tensor(a!) parts, Tensor(b!) part_rows) -> ()");
  m.def(
      "vae_sample_forward_(int B, int Z, float v_pm, float v_pv, float v_plv, Tensor mu, "
      "Tensor lv, Tensor eps, Tensor(a!) z, Tensor(b!)? z_bf16, int ld_zb, Tensor act, "
      "Tensor(c!)? runloss, Tensor(d!) vkl) -> ()");
  m.def(
      "air_runloss_(int T, int B, Tensor(b!) rec, int rec_step_stride, Tensor skl, Tensor shkl, "
      "Tensor vkl, Tensor(a!) runloss, Tensor? live=None) -> ()");
  m.def(
      "vae_sample_backward_(int B, int Z, float v_pm, float v_pv, float grad_scale, Tensor mu, "
      "Tensor lv, Tensor eps, Tensor dz, Tensor act, Tensor(a!)? dmu, Tensor(b!)? dlv, "
      "Tensor(c!)? dmu_bf16, Tensor(d!)? dlv_bf16, int ld_b) -> ()");
  m.def("sigmoid_backward_(Tensor r, Tensor dr, Tensor(a!) dm, int n) -> ()");
  m.def(
      "stn_vae_step_(int B, int C, Tensor x, Tensor theta_f, Tensor theta_b, Tensor mask, "
      "Tensor zval, Tensor eps_z, Tensor? eps_x, int eps_seed, int eps_offset, bool eps_gen, "
      "Tensor[] wt, Tensor[] bias, float lik_std, float v_pm, float v_pv, float v_plv, "
      "Tensor(a!) canvas_part, Tensor(b!) part_rows, Tensor(c!)? runloss, Tensor(d!) vkl, "
      "Tensor(e!)? gb, Tensor(f!)? a1b, Tensor(g!)? a2b, Tensor(h!)? mu, Tensor(i!)? lv, "
      "Tensor(j!)? z, Tensor(k!)? zb, Tensor(l!)? d1b, Tensor(m!)? d2b, Tensor(n!) r, "
      "int x_period=0) -> ()");
  m.def("pack_frag_f32_(Tensor[] W, int[] K, int[] N, Tensor(a!)?[] out) -> ()");
  m.def(
      "stn_vae_step_f32_(int B, int C, Tensor x, Tensor theta_f, Tensor theta_b, Tensor mask, "
      "Tensor zval, Tensor eps_z, Tensor? eps_x, int eps_seed, int eps_offset, bool eps_gen, "
      "Tensor[] wt, Tensor[] bias, float lik_std, float v_pm, float v_pv, float v_plv, "
      "Tensor(a!) canvas_part, Tensor(b!) part_rows, Tensor(c!)? runloss, Tensor(d!) vkl, "
      "Tensor(e!)?[] saved, Tensor(f!) z, Tensor(g!) r, int x_period=0) -> ()");
  m.def(
      "recon_loss_(Tensor x, Tensor(a!)? canvas, Tensor? parts, int nparts, int part_stride, "
      "Tensor? part_rows, int C, Tensor runloss, Tensor digits, Tensor? targets, int B, int C2, "
      "float grad_scale, Tensor(b!)? recon, Tensor(c!) bce, Tensor(d!) mse, Tensor(e!) loss, "
      "Tensor(f!)? acc, Tensor(g!)? dcanvas) -> ()");
  m.def(
      "batch_mean_(Tensor? a0, Tensor? a1, Tensor? a2, Tensor? a3, int B, Tensor(a!) out) -> ()");
  m.def(
      "clip_adam_(Tensor(a!) params, Tensor(b!) grads, Tensor(c!) m, Tensor(d!) v, Tensor off, "
      "Tensor len, Tensor block_tensor, Tensor block_start, int nblocks, Tensor(e!)? sumsq, "
      "float clip, float lr_t, float beta1, float beta2, float eps) -> ()");
  m.def("add_(Tensor a, Tensor b, Tensor(a!) out, int n) -> ()");
  m.def("rng_fill_(Tensor(a!) out, int seed, int offset, bool normal) -> ()");
  m.def("rng_fill_batch_(Tensor(a!)[] out, int seed, int[] offset, int[] normal) -> ()");
  m.def("fill32_batch_(Tensor(a!)[] dst, int[] value) -> ()");
  m.def("copy_f4_(Tensor src, Tensor(a!) dst) -> ()");
  // AIR-ASR (air_number_bbox_location.py:384-1084)
  m.def(
      "asr_pack_(int B, int Z, int H, int ld, Tensor? z, Tensor? ss, Tensor? h, "
      "Tensor(a!) out, Tensor? h2=None, Tensor(b!)? out2=None) -> ()");
  m.def(
      "asr_unpack_(int B, int Z, int H, int ld, Tensor dU, Tensor dUg, Tensor(a!) dz, "
      "Tensor(b!) dss, Tensor(c!) dh, Tensor(d!) dhg, int acc_dz=0) -> ()");
  m.def(
      "asr_step_forward_(int B, int step, bool train, int fix_steps, float thr, "
      "float temperature, float s_pm, float s_pv, float s_plv, float gamma_num, Tensor[] w, "
      "Tensor(a!)?[] hid, Tensor eps_shift, Tensor eps_scale, Tensor u, Tensor(b!) stop, "
      "Tensor(c!) digits, Tensor(d!) live, Tensor(e!) rec, Tensor(f!) theta_fwd, "
      "Tensor(g!) theta_back, Tensor(h!) ss, Tensor(i!) scale, Tensor(j!) shift, "
      "Tensor(k!) zprob, Tensor(l!) zmask, Tensor(m!) zval, Tensor(n!) zc) -> ()");
  m.def(
      "asr_terms_(int B, int T, int C, int[] cons, float[] gammas, Tensor rec, Tensor vkl, "
      "Tensor zmask, Tensor live, Tensor(a!) klsum, Tensor(b!) pr, Tensor(c!) area, "
      "Tensor(d!) out, Tensor(e!) size, Tensor(f!) overlap, Tensor(g!) zsum) -> ()");
  m.def(
      "asr_finalize_(int B, int T, int C, int[] cons, float[] gammas, float inv_batch_global, "
      "Tensor rec, Tensor live, Tensor zsum, Tensor pr, Tensor(a!) loss, Tensor(b!) element, "
      "Tensor(c!) margin) -> ()");
  m.def(
      "asr_terms_backward_(int B, int T, int C, int[] cons, float[] gammas, float grad_scale, "
      "float inv_batch_global, Tensor rec, Tensor live, Tensor zsum, Tensor(a!) dreg) -> ()");
  m.def(
      "asr_step_backward_(int B, bool train, int fix_steps, float temperature, float s_pm, "
      "float s_pv, float grad_scale, Tensor[] w, Tensor?[] hid, Tensor rec, Tensor eps_shift, "
      "Tensor eps_scale, Tensor dtheta_fwd, Tensor dtheta_back, Tensor dot, Tensor dreg, "
      "Tensor? dss, Tensor(a!) douts, Tensor(b!)?[] dpre) -> ()");
}

TORCH_LIBRARY_IMPL(mog_air, CUDA, m) {
  m.impl("gemm_f32_", &gemm_f32_);
  m.impl("gemm_f32_kseg_", &gemm_f32_kseg_);
  m.impl("gemm_f32_sigmoid_philox_", &gemm_f32_sigmoid_philox_);
  m.impl("gemm_f32_x3_tn_", &gemm_f32_x3_tn_);
  m.impl("split3_bf16_", &split3_bf16_);
  m.impl("gemm_x3_nt_", &gemm_x3_nt_);
  m.impl("gemm_x3p_tn_", &gemm_x3p_tn_);
  m.impl("gemm_f32_wgrad_group_", &gemm_f32_wgrad_group_);
  m.impl("wgrad_tn_bf16_", &wgrad_tn_bf16_);
  m.impl("wgrad_tn_x3_", &wgrad_tn_x3_);
  m.impl("gemm_bf16_", &gemm_bf16_);
  m.impl("cvt_bf16_batch_", &cvt_bf16_batch_);
  m.impl("stn_forward_", &stn_forward_);
  m.impl("stn_backward_", &stn_backward_);
  m.impl("stn_backward_sigmoid_", &stn_backward_sigmoid_);
  m.impl("lstm_cell_forward_", &lstm_cell_forward_);
  m.impl("lstm_cell_backward_", &lstm_cell_backward_);
  m.impl("gemm_f32_kseg_group_", &gemm_f32_kseg_group_);
  m.impl("lstm_cell_forward2_", &lstm_cell_forward2_);
  m.impl("lstm_cell_backward2_", &lstm_cell_backward2_);
  m.impl("heads_output_wgrad_", &heads_output_wgrad_);
  m.impl("split3_sum_bf16_", &split3_sum_bf16_);
  m.impl("lstm_cell_backward_parts_", &lstm_cell_backward_parts_);
  m.impl("asr_unpack_parts_", &asr_unpack_parts_);
  m.impl("copy32_batch_", &copy32_batch_);
  m.impl("transpose32_batch_", &transpose32_batch_);
  m.impl("air_step_forward_", &air_step_forward_);
  m.impl("air_step_forward_steps_", &air_step_forward_steps_);
  m.impl("air_step_backward_", &air_step_backward_);
  m.impl("generation_prior_", &generation_prior_);
  m.impl("vae_sample_forward_", &vae_sample_forward_);
  m.impl("vae_sample_backward_", &vae_sample_backward_);
  m.impl("air_runloss_", &air_runloss_);
  m.impl("stn_write_parts_", &stn_write_parts_);
  m.impl("sigmoid_backward_", &sigmoid_backward_);
  m.impl("stn_vae_step_", &stn_vae_step_);
  m.impl("pack_frag_f32_", &pack_frag_f32_);
  m.impl("stn_vae_step_f32_", &stn_vae_step_f32_);
  m.impl("recon_loss_", &recon_loss_);
  m.impl("batch_mean_", &batch_mean_);
  m.impl("clip_adam_", &clip_adam_);
  m.impl("add_", &add_);
  m.impl("rng_fill_", &rng_fill_);
  m.impl("rng_fill_batch_", &rng_fill_batch_);
  m.impl("fill32_batch_", &fill32_batch_);
  m.impl("copy_f4_", &copy_f4_);
  m.impl("asr_pack_", &asr_pack_);
  m.impl("asr_unpack_", &asr_unpack_);
  m.impl("asr_step_forward_", &asr_step_forward_);
  m.impl("asr_terms_", &asr_terms_);
  m.impl("asr_finalize_", &asr_finalize_);
  m.impl("asr_terms_backward_", &asr_terms_backward_);
  m.impl("asr_step_backward_", &asr_step_backward_);
}
