// PyTorch-ROCm custom operators over the C ABI of libmog_air.so
// (include/mog_air.h): TORCH_LIBRARY_FRAGMENT(mog_air) schemas with HIP
// (dispatch key CUDA on ROCm) implementations, so the Python host drives every
// hot-path launch through torch.ops.mog_air.* (SURVEY.md §8 B).  Each op takes
// device tensors (or views: a tensor's data_ptr is the matrix origin) and plain
// scalars, launches on torch's current HIP stream, and raises (c10::Error ->
// RuntimeError) when the C ABI rejects an argument.  There is no CPU kernel: a
// CPU tensor finds no implementation and fails loudly.
//
// The ops are the launch-level (mutating, "out=") form the AIRModel schedules
// its forward / backward with; differentiable functional ops built on them
// live in mog_air/torch_ops.py.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "mog_air.h"

namespace {

using at::Tensor;
using c10::optional;
using std::vector;

void* stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* name) {
  TORCH_CHECK(rc == 0, "mog_air::", name, " failed: ",
              rc == MOG_ERR_INVALID ? "invalid argument" : "HIP error ", rc);
}

void* p(const Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "mog_air ops take HIP device tensors (no CPU implementation)");
  return t.data_ptr();
}
void* p(const optional<Tensor>& t) { return t.has_value() && t->defined() ? p(*t) : nullptr; }
float* f(const Tensor& t) { return static_cast<float*>(p(t)); }
float* f(const optional<Tensor>& t) { return static_cast<float*>(p(t)); }

// device pointer arrays of tensor lists (None entries -> NULL)
vector<void*> ptrs(const at::TensorList& ts) {
  vector<void*> v;
  for (const auto& t : ts) v.push_back(p(t));
  return v;
}
vector<void*> ptrs(const c10::List<optional<Tensor>>& ts) {
  vector<void*> v;
  for (size_t i = 0; i < ts.size(); ++i) v.push_back(p(static_cast<optional<Tensor>>(ts[i])));
  return v;
}
template <class T>
const T* const* arr(const vector<void*>& v) {
  return v.empty() ? nullptr : reinterpret_cast<const T* const*>(v.data());
}
template <class T>
T* const* marr(const vector<void*>& v) {
  return v.empty() ? nullptr : reinterpret_cast<T* const*>(v.data());
}

// ---------------------------------------------------------------- GEMMs ----
void gemm_f32_(at::TensorList A, at::TensorList B, at::TensorList C,
               const c10::List<optional<Tensor>>& bias, const c10::List<optional<Tensor>>& Cin,
               const c10::List<optional<Tensor>>& Cpre, const c10::List<optional<Tensor>>& aux,
               const c10::List<optional<Tensor>>& colsum, int64_t M, int64_t N, int64_t K,
               int64_t lda, int64_t ldb, int64_t ldc, int64_t ldaux, bool transA, bool transB,
               int64_t epi, double aux_scale, int64_t splitk) {
  auto a = ptrs(A), b = ptrs(B), c = ptrs(C), bi = ptrs(bias), ci = ptrs(Cin), cp = ptrs(Cpre),
       ax = ptrs(aux), cs = ptrs(colsum);
  check(mog_gemm_f32((int)c.size(), arr<float>(a), arr<float>(b), marr<float>(c), arr<float>(bi),
                     arr<float>(ci), marr<float>(cp), arr<float>(ax), marr<float>(cs), M, N, K, lda,
                     ldb, ldc, ldaux, transA, transB, epi, (float)aux_scale, splitk, stream()),
        "gemm_f32_");
}

void gemm_f32_sigmoid_philox_(const Tensor& A, const Tensor& B, Tensor C,
                              const optional<Tensor>& bias, int64_t M, int64_t N, int64_t K,
                              int64_t lda, int64_t ldb, int64_t ldc, double scale, int64_t seed,
                              int64_t offset) {
  check(mog_gemm_f32_sigmoid_philox(f(A), f(B), f(C), f(bias), M, N, K, lda, ldb, ldc,
                                    (float)scale, (unsigned long long)seed,
                                    (unsigned long long)offset, stream()),
        "gemm_f32_sigmoid_philox_");
}

void gemm_f32_kseg_(at::TensorList A, at::TensorList B, Tensor C, const optional<Tensor>& bias,
                    const optional<Tensor>& Cin, int64_t M, int64_t N, int64_t kseg, int64_t lda,
                    int64_t ldb, int64_t ldc, bool transA, bool transB, int64_t epi) {
  auto a = ptrs(A), b = ptrs(B);
  check(mog_gemm_f32_kseg((int)a.size(), arr<float>(a), arr<float>(b), f(C), f(bias), f(Cin), M, N,
                          kseg, lda, ldb, ldc, transA, transB, epi, stream()),
        "gemm_f32_kseg_");
}

void gemm_bf16_(at::TensorList A, at::TensorList B, at::TensorList C,
                const c10::List<optional<Tensor>>& bias, const c10::List<optional<Tensor>>& Cin,
                const c10::List<optional<Tensor>>& aux, const c10::List<optional<Tensor>>& colsum,
                int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                int64_t ldaux, bool tn, int64_t epi, double aux_scale, int64_t splitk) {
  auto a = ptrs(A), b = ptrs(B), c = ptrs(C), bi = ptrs(bias), ci = ptrs(Cin), ax = ptrs(aux),
       cs = ptrs(colsum);
  const bool out_bf16 = C.size() > 0 && C[0].scalar_type() == at::kBFloat16;
  check(mog_gemm_bf16((int)c.size(), arr<void>(a), arr<void>(b), marr<void>(c), arr<float>(bi),
                      arr<float>(ci), arr<void>(ax), marr<float>(cs), M, N, K, lda, ldb, ldc,
                      ldaux, tn, epi, out_bf16, (float)aux_scale, splitk, stream()),
        "gemm_bf16_");
}

void cvt_bf16_batch_(at::TensorList src, at::TensorList dst, at::IntArrayRef dims) {
  auto s = ptrs(src), d = ptrs(dst);
  vector<int> di(dims.begin(), dims.end());
  TORCH_CHECK(di.size() == 7 * s.size() && s.size() == d.size(), "cvt_bf16_batch_: 7 dims per job");
  check(mog_cvt_bf16_batch((int)s.size(), arr<float>(s), marr<void>(d), di.data(), stream()),
        "cvt_bf16_batch_");
}

// ------------------------------------------------------------------ STN ----
void stn_forward_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win, const Tensor& theta,
                  int64_t Hout, int64_t Wout, Tensor out, const optional<Tensor>& z,
                  const optional<Tensor>& mask, int64_t mode) {
  check(mog_stn_forward(f(U), N, Hin, Win, f(theta), Hout, Wout, p(out), f(z), f(mask), mode,
                        stream()),
        "stn_forward_");
}

void stn_backward_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win, const Tensor& theta,
                   int64_t Hout, int64_t Wout, const Tensor& G, const optional<Tensor>& gscale,
                   const optional<Tensor>& dU, const optional<Tensor>& dtheta,
                   const optional<Tensor>& dot, int64_t u_period, int64_t g_period) {
  check(mog_stn_backward(f(U), N, Hin, Win, f(theta), Hout, Wout, f(G), f(gscale), f(dU),
                         f(dtheta), f(dot), u_period, g_period, stream()),
        "stn_backward_");
}

void stn_backward_sigmoid_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win,
                                const Tensor& theta, int64_t Hout, int64_t Wout, const Tensor& G,
                                const optional<Tensor>& gscale, Tensor dm,
                                const optional<Tensor>& dtheta, const optional<Tensor>& dot,
                                int64_t g_period) {
  // dm bf16 (configs[1]) or fp32 (reference precision)
  if (dm.scalar_type() == at::kBFloat16)
    check(mog_stn_backward_sigmoid_bf16(f(U), N, Hin, Win, f(theta), Hout, Wout, f(G), f(gscale),
                                        p(dm), f(dtheta), f(dot), 0, g_period, stream()),
          "stn_backward_sigmoid_");
  else
    check(mog_stn_backward_sigmoid_f32(f(U), N, Hin, Win, f(theta), Hout, Wout, f(G), f(gscale),
                                       f(dm), f(dtheta), f(dot), 0, g_period, stream()),
          "stn_backward_sigmoid_");
}

// ----------------------------------------------------------------- LSTM ----
void lstm_cell_forward_(const Tensor& G, const optional<Tensor>& bias,
                        const optional<Tensor>& c_prev, Tensor c_out, Tensor h_out, int64_t B,
                        int64_t H) {
  check(mog_lstm_cell_forward(f(G), f(bias), f(c_prev), f(c_out), f(h_out), B, H, stream()),
        "lstm_cell_forward_");
}

void lstm_cell_backward_(const Tensor& G, const optional<Tensor>& bias,
                         const optional<Tensor>& c_prev, const Tensor& c_cur, const Tensor& dh,
                         const optional<Tensor>& dc, Tensor dG, Tensor dc_prev,
                         const optional<Tensor>& dGsum, int64_t B, int64_t H) {
  check(mog_lstm_cell_backward(f(G), f(bias), f(c_prev), f(c_cur), f(dh), f(dc), f(dG),
                               f(dc_prev), f(dGsum), B, H, stream()),
        "lstm_cell_backward_");
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
                       Tensor zc) {
  auto h = ptrs(hid), w = ptrs(w2), b = ptrs(b2);
  TORCH_CHECK(h.size() == 5 && w.size() == 5 && b.size() == 5, "air_step_forward_: 5 heads");
  check(mog_air_step_forward(B, HS, HZ, step, train, use_num_prior, thr, temperature, prior_lo,
                             prior_bias, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv, arr<float>(h),
                             arr<float>(w), arr<float>(b), f(eps_scale), f(eps_shift), f(u),
                             f(stop), f(runloss), static_cast<int*>(p(digits)),
                             static_cast<int*>(p(live)), f(rec), f(theta_fwd), f(theta_back),
                             f(scale), f(shift), f(zprob), f(zkl), f(skl), f(shkl), f(zmask),
                             f(zval), f(zc), stream()),
        "air_step_forward_");
}

void air_step_backward_(int64_t B, int64_t HS, bool train, bool use_num_prior,
                        double temperature, double prior_lo, double prior_bias, double s_pm,
                        double s_pv, double h_pm, double h_pv, double grad_scale,
                        const optional<Tensor>& dloss, const Tensor& rec, const Tensor& eps_scale, const Tensor& eps_shift,
                        const Tensor& dtheta_fwd, const Tensor& dtheta_back, const Tensor& dot,
                        at::TensorList hid, at::TensorList w2, Tensor dout, int64_t dout_hs,
                        Tensor dhid, int64_t dhid_hs) {
  auto h = ptrs(hid), w = ptrs(w2);
  TORCH_CHECK(h.size() == 5 && w.size() == 5, "air_step_backward_: 5 heads");
  check(mog_air_step_backward(B, HS, train, use_num_prior, temperature, prior_lo, prior_bias, s_pm,
                              s_pv, h_pm, h_pv, grad_scale, f(dloss), f(rec),
                              f(eps_scale), f(eps_shift),
                              f(dtheta_fwd), f(dtheta_back), f(dot), arr<float>(h), arr<float>(w),
                              f(dout), dout_hs, f(dhid), dhid_hs, stream()),
        "air_step_backward_");
}

void stn_write_parts_(const Tensor& U, int64_t N, int64_t Hin, int64_t Win, const Tensor& theta,
                      int64_t Hout, int64_t Wout, const Tensor& z, const Tensor& mask, Tensor parts,
                      Tensor part_rows) {
  check(mog_stn_write_parts(f(U), N, Hin, Win, f(theta), Hout, Wout, f(z), f(mask), f(parts),
                            static_cast<int*>(p(part_rows)), stream()),
        "stn_write_parts_");
}

// ------------------------------------------------------------ glimpse VAE ----
void vae_sample_forward_(int64_t B, int64_t Z, double v_pm, double v_pv, double v_plv,
                         const Tensor& mu, const Tensor& lv, const Tensor& eps, Tensor z,
                         const optional<Tensor>& z_bf16, int64_t ld_zb, const Tensor& act,
                         const optional<Tensor>& runloss, Tensor vkl) {
  check(mog_vae_sample_forward(B, Z, v_pm, v_pv, v_plv, f(mu), f(lv), f(eps), f(z), p(z_bf16),
                               ld_zb, f(act), f(runloss), f(vkl), stream()),
        "vae_sample_forward_");
}

void air_runloss_(int64_t T, int64_t B, const Tensor& rec, int64_t rec_step_stride,
                  const Tensor& skl, const Tensor& shkl, const Tensor& vkl, Tensor runloss) {
  check(mog_air_runloss(T, B, f(rec), rec_step_stride, f(skl), f(shkl), f(vkl), f(runloss),
                        stream()),
        "air_runloss_");
}

void vae_sample_backward_(int64_t B, int64_t Z, double v_pm, double v_pv, double grad_scale,
                          const Tensor& mu, const Tensor& lv, const Tensor& eps, const Tensor& dz,
                          const Tensor& act, const optional<Tensor>& dmu,
                          const optional<Tensor>& dlv, const optional<Tensor>& dmu_bf16,
                          const optional<Tensor>& dlv_bf16, int64_t ld_b) {
  check(mog_vae_sample_backward(B, Z, v_pm, v_pv, grad_scale, f(mu), f(lv), f(eps), f(dz), f(act),
                                f(dmu), f(dlv), p(dmu_bf16), p(dlv_bf16), ld_b, stream()),
        "vae_sample_backward_");
}

void sigmoid_backward_(const Tensor& r, const Tensor& dr, Tensor dm, int64_t n) {
  check(mog_sigmoid_backward(f(r), f(dr), p(dm), n, dm.scalar_type() == at::kBFloat16, stream()),
        "sigmoid_backward_");
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
  auto w = ptrs(wt), b = ptrs(bias);
  TORCH_CHECK(w.size() == 7 && b.size() == 7, "stn_vae_step_: 7 VAE layers");
  check(mog_stn_vae_step_forward(B, C, 28, 512, 256, 50, 256, 512, f(x), f(theta_f), f(theta_b),
                                 f(mask), f(zval), f(eps_z), f(eps_x), eps_gen,
                                 (unsigned long long)eps_seed, (unsigned long long)eps_offset,
                                 arr<void>(w), arr<float>(b), lik_std, v_pm, v_pv, v_plv,
                                 f(canvas_part), static_cast<int*>(p(part_rows)), f(runloss),
                                 f(vkl), p(gb), p(a1b), p(a2b), f(mu), f(lv), f(z), p(zb), p(d1b),
                                 p(d2b), f(r), x_period, stream()),
        "stn_vae_step_");
}

// ------------------------------------------------- loss / optimizer / RNG ----
void recon_loss_(const Tensor& x, const optional<Tensor>& canvas, const optional<Tensor>& parts,
                 int64_t nparts, int64_t part_stride, const optional<Tensor>& part_rows, int64_t C,
                 const Tensor& runloss, const Tensor& digits, const optional<Tensor>& targets,
                 int64_t B, int64_t C2, double grad_scale, const optional<Tensor>& recon,
                 Tensor bce, Tensor mse, Tensor loss, const optional<Tensor>& acc,
                 const optional<Tensor>& dcanvas) {
  check(mog_recon_loss(f(x), f(canvas), f(parts), nparts, part_stride,
                       static_cast<const int*>(p(part_rows)), C, f(runloss),
                       static_cast<const int*>(p(digits)), static_cast<const int*>(p(targets)), B,
                       C2, grad_scale, f(recon), f(bce), f(mse), f(loss), f(acc), f(dcanvas),
                       stream()),
        "recon_loss_");
}

void batch_mean_(const optional<Tensor>& a0, const optional<Tensor>& a1,
                 const optional<Tensor>& a2, const optional<Tensor>& a3, int64_t B, Tensor out) {
  check(mog_batch_mean(f(a0), f(a1), f(a2), f(a3), B, f(out), stream()), "batch_mean_");
}

void clip_adam_(Tensor params, Tensor grads, Tensor m, Tensor v, const Tensor& off,
                const Tensor& len, const Tensor& block_tensor, const Tensor& block_start,
                int64_t nblocks, const optional<Tensor>& sumsq, double clip, double lr_t,
                double beta1, double beta2, double eps) {
  check(mog_clip_adam(f(params), f(grads), f(m), f(v), static_cast<const long*>(p(off)),
                      static_cast<const long*>(p(len)), static_cast<const int*>(p(block_tensor)),
                      static_cast<const long*>(p(block_start)), nblocks, f(sumsq), clip, lr_t,
                      beta1, beta2, eps, stream()),
        "clip_adam_");
}

void add_(const Tensor& a, const Tensor& b, Tensor out, int64_t n) {
  check(mog_add(f(a), f(b), f(out), n, stream()), "add_");
}

void rng_fill_(Tensor out, int64_t seed, int64_t offset, bool normal) {
  check(mog_rng_fill(f(out), out.numel(), (unsigned long long)seed, (unsigned long long)offset,
                     normal, stream()),
        "rng_fill_");
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(mog_air, m) {
  m.def(
      "gemm_f32_(Tensor[] A, Tensor[] B, Tensor(a!)[] C, Tensor?[] bias, Tensor?[] Cin, "
      "Tensor?[] Cpre, Tensor?[] aux, Tensor?[] colsum, int M, int N, int K, int lda, int ldb, "
      "int ldc, int ldaux, bool transA, bool transB, int epi, float aux_scale, int splitk) -> ()");
  m.def(
      "gemm_f32_sigmoid_philox_(Tensor A, Tensor B, Tensor(a!) C, Tensor? bias, int M, int N, "
      "int K, int lda, int ldb, int ldc, float scale, int seed, int offset) -> ()");
  m.def(
      "gemm_f32_kseg_(Tensor[] A, Tensor[] B, Tensor(a!) C, Tensor? bias, Tensor? Cin, int M, "
      "int N, int kseg, int lda, int ldb, int ldc, bool transA, bool transB, int epi) -> ()");
  m.def(
      "gemm_bf16_(Tensor[] A, Tensor[] B, Tensor(a!)[] C, Tensor?[] bias, Tensor?[] Cin, "
      "Tensor?[] aux, Tensor?[] colsum, int M, int N, int K, int lda, int ldb, int ldc, "
      "int ldaux, bool tn, int epi, float aux_scale, int splitk) -> ()");
  m.def("cvt_bf16_batch_(Tensor[] src, Tensor(a!)[] dst, int[] dims) -> ()");
  m.def(
      "stn_forward_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, int Wout, "
      "Tensor(a!) out, Tensor? z, Tensor? mask, int mode) -> ()");
  m.def(
      "stn_backward_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, int Wout, "
      "Tensor G, Tensor? gscale, Tensor? dU, Tensor? dtheta, Tensor? dot, int u_period, "
      "int g_period) -> ()");
  m.def(
      "stn_backward_sigmoid_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, "
      "int Wout, Tensor G, Tensor? gscale, Tensor(a!) dm, Tensor? dtheta, Tensor? dot, "
      "int g_period) -> ()");
  m.def(
      "lstm_cell_forward_(Tensor G, Tensor? bias, Tensor? c_prev, Tensor(a!) c_out, "
      "Tensor(b!) h_out, int B, int H) -> ()");
  m.def(
      "lstm_cell_backward_(Tensor G, Tensor? bias, Tensor? c_prev, Tensor c_cur, Tensor dh, "
      "Tensor? dc, Tensor(a!) dG, Tensor(b!) dc_prev, Tensor? dGsum, int B, int H) -> ()");
  m.def(
      "air_step_forward_(int B, int HS, int HZ, int step, bool train, bool use_num_prior, "
      "float thr, float temperature, float prior_lo, float prior_bias, float s_pm, float s_pv, "
      "float s_plv, float h_pm, float h_pv, float h_plv, Tensor[] hid, Tensor[] w2, "
      "Tensor[] b2, Tensor eps_scale, Tensor eps_shift, Tensor u, Tensor(a!) stop, "
      "Tensor(b!) runloss, Tensor(c!) digits, Tensor(d!) live, Tensor(e!) rec, "
      "Tensor(f!) theta_fwd, Tensor(g!) theta_back, Tensor(h!) scale, Tensor(i!) shift, "
      "Tensor(j!) zprob, Tensor(k!) zkl, Tensor(l!) skl, Tensor(m!) shkl, Tensor(n!) zmask, "
      "Tensor(o!) zval, Tensor(p!) zc) -> ()");
  m.def(
      "air_step_backward_(int B, int HS, bool train, bool use_num_prior, float temperature, "
      "float prior_lo, float prior_bias, float s_pm, float s_pv, float h_pm, float h_pv, "
      "float grad_scale, Tensor? dloss, Tensor rec, Tensor eps_scale, Tensor eps_shift, "
      "Tensor dtheta_fwd, "
      "Tensor dtheta_back, Tensor dot, Tensor[] hid, Tensor[] w2, Tensor(a!) dout, int dout_hs, "
      "Tensor(b!) dhid, int dhid_hs) -> ()");
  m.def(
      "stn_write_parts_(Tensor U, int N, int Hin, int Win, Tensor theta, int Hout, int Wout, "
      "Tensor z, Tensor mask, Tensor(a!) parts, Tensor(b!) part_rows) -> ()");
  m.def(
      "vae_sample_forward_(int B, int Z, float v_pm, float v_pv, float v_plv, Tensor mu, "
      "Tensor lv, Tensor eps, Tensor(a!) z, Tensor? z_bf16, int ld_zb, Tensor act, "
      "Tensor(b!)? runloss, Tensor(c!) vkl) -> ()");
  m.def(
      "air_runloss_(int T, int B, Tensor rec, int rec_step_stride, Tensor skl, Tensor shkl, "
      "Tensor vkl, Tensor(a!) runloss) -> ()");
  m.def(
      "vae_sample_backward_(int B, int Z, float v_pm, float v_pv, float grad_scale, Tensor mu, "
      "Tensor lv, Tensor eps, Tensor dz, Tensor act, Tensor? dmu, Tensor? dlv, Tensor? dmu_bf16, "
      "Tensor? dlv_bf16, int ld_b) -> ()");
  m.def("sigmoid_backward_(Tensor r, Tensor dr, Tensor(a!) dm, int n) -> ()");
  m.def(
      "stn_vae_step_(int B, int C, Tensor x, Tensor theta_f, Tensor theta_b, Tensor mask, "
      "Tensor zval, Tensor eps_z, Tensor? eps_x, int eps_seed, int eps_offset, bool eps_gen, "
      "Tensor[] wt, Tensor[] bias, float lik_std, float v_pm, float v_pv, float v_plv, "
      "Tensor(a!) canvas_part, Tensor(b!) part_rows, Tensor(c!)? runloss, Tensor(d!) vkl, "
      "Tensor(e!)? gb, Tensor(f!)? a1b, Tensor(g!)? a2b, Tensor(h!)? mu, Tensor(i!)? lv, "
      "Tensor(j!)? z, Tensor(k!)? zb, Tensor(l!)? d1b, Tensor(m!)? d2b, Tensor(n!) r, "
      "int x_period=0) -> ()");
  m.def(
      "recon_loss_(Tensor x, Tensor? canvas, Tensor? parts, int nparts, int part_stride, "
      "Tensor? part_rows, int C, Tensor runloss, Tensor digits, Tensor? targets, int B, int C2, "
      "float grad_scale, Tensor? recon, Tensor(a!) bce, Tensor(b!) mse, Tensor(c!) loss, "
      "Tensor? acc, Tensor? dcanvas) -> ()");
  m.def(
      "batch_mean_(Tensor? a0, Tensor? a1, Tensor? a2, Tensor? a3, int B, Tensor(a!) out) -> ()");
  m.def(
      "clip_adam_(Tensor(a!) params, Tensor(b!) grads, Tensor(c!) m, Tensor(d!) v, Tensor off, "
      "Tensor len, Tensor block_tensor, Tensor block_start, int nblocks, Tensor? sumsq, "
      "float clip, float lr_t, float beta1, float beta2, float eps) -> ()");
  m.def("add_(Tensor a, Tensor b, Tensor(a!) out, int n) -> ()");
  m.def("rng_fill_(Tensor(a!) out, int seed, int offset, bool normal) -> ()");
}

TORCH_LIBRARY_IMPL(mog_air, CUDA, m) {
  m.impl("gemm_f32_", &gemm_f32_);
  m.impl("gemm_f32_kseg_", &gemm_f32_kseg_);
  m.impl("gemm_f32_sigmoid_philox_", &gemm_f32_sigmoid_philox_);
  m.impl("gemm_bf16_", &gemm_bf16_);
  m.impl("cvt_bf16_batch_", &cvt_bf16_batch_);
  m.impl("stn_forward_", &stn_forward_);
  m.impl("stn_backward_", &stn_backward_);
  m.impl("stn_backward_sigmoid_", &stn_backward_sigmoid_);
  m.impl("lstm_cell_forward_", &lstm_cell_forward_);
  m.impl("lstm_cell_backward_", &lstm_cell_backward_);
  m.impl("air_step_forward_", &air_step_forward_);
  m.impl("air_step_backward_", &air_step_backward_);
  m.impl("vae_sample_forward_", &vae_sample_forward_);
  m.impl("vae_sample_backward_", &vae_sample_backward_);
  m.impl("air_runloss_", &air_runloss_);
  m.impl("stn_write_parts_", &stn_write_parts_);
  m.impl("sigmoid_backward_", &sigmoid_backward_);
  m.impl("stn_vae_step_", &stn_vae_step_);
  m.impl("recon_loss_", &recon_loss_);
  m.impl("batch_mean_", &batch_mean_);
  m.impl("clip_adam_", &clip_adam_);
  m.impl("add_", &add_);
  m.impl("rng_fill_", &rng_fill_);
}
