/*
 * mog_air.h — C ABI of the MI355X-native AIR hot path (libmog_air.so).
 *
 * Plain pointers and sizes only: every float / int pointer is DEVICE memory
 * (HBM of the current HIP device) unless stated otherwise, `stream` is a
 * hipStream_t passed as void*.  Every entry point is asynchronous on `stream`
 * and returns 0 on success, MOG_ERR_INVALID (1001) for a rejected argument, or
 * a hipError_t code from the launch.  No entry point allocates, frees or
 * synchronises, so any sequence of calls can be captured into a hipGraph.
 *
 * The reference (taufikxu/MOG-ASR) is Python/TF-1.12 with no FFI; each entry
 * point below names the reference interface (file:line) whose behaviour it
 * replaces.  INTEGRATION.md shows the ctypes binding used by the Python host
 * (mog-asr_amd/mog_air/_lib.py).
 */
#ifndef MOG_AIR_H
#define MOG_AIR_H

#ifdef __cplusplus
extern "C" {
#endif

#define MOG_ERR_INVALID 1001

/* ---- dense layers / matmul ------------------------------------------------
 * Replaces tf.matmul + bias_add + activation of contrib.layers.fully_connected
 * (air/vae.py:18-41, air/air_model.py:462-499,596-600), the LSTM kernel matmul
 * (air_model.py:454-456, TF BasicLSTMCell) and their gradients.
 * Batched over `batch` (<= 8) problems given as HOST arrays of device
 * pointers.  A(m,k) = transA ? A[k*lda+m] : A[m*lda+k]; B likewise.
 * epi: 0 store(+bias) 1 relu 2 softplus(TF) 3 sigmoid(acc+bias+aux*aux_scale)
 *      4 acc*(1-exp(-aux)) [= acc*sigmoid(x), aux = softplus(x), the layer's
 *      output] 5 atomic-add 6 relu-backward (aux = activation).
 * With splitk == 1 every output is one k-ordered fp32 fma chain (bit-exact
 * with the oracle).  splitk > 1 requires epi 5.  colsum (epi 5 only, may be
 * NULL): colsum[z][n] += sum_k B_z(k, n) — the bias gradient of a weight-
 * gradient GEMM dW = X^T dY (TF BiasAddGrad), fused. */
int mog_gemm_f32(int batch, const float* const* A, const float* const* B, float* const* C,
                 const float* const* bias, const float* const* Cin, float* const* Cpre,
                 const float* const* aux, float* const* colsum, int M, int N, int K, int lda,
                 int ldb, int ldc, int ldaux, int transA, int transB, int epi, float aux_scale,
                 int splitk, void* stream);

/* fp32 weight gradient on the bf16 matrix cores (mog-asr_amd/csrc/gemm_x3.hip):
 * C[m][n] += sum_k A[k*lda+m] B[k*ldb+n] over `splitk` k-ranges, colsum[n] +=
 * sum_k B[k*ldb+n] when colsum != NULL.  Split-K partials: with `work` (>=
 * splitk * M * N floats, + splitk * N with a colsum) each range's product and
 * column sums are stored there and a second launch adds the ranges into C and
 * colsum in a fixed order (deterministic; plain stores instead of float
 * atomics, which run at about 1.3 TB/s); work == NULL: float atomics.  One k-range: C += product by a plain read-add-write.  Each fp32 operand is split
 * exactly into three bf16 pieces; the six products down to 2^-16 relative are
 * accumulated in fp32 (error of the order of one fp32 product rounding; not a
 * k-ordered chain, so tolerance-gated like every split-K gradient).  The x-part
 * of the LSTM kernel gradient (TF MatMul gradient of air_model.py:454-456).
 * A, B 16-byte aligned; M, N, lda, ldb multiples of 4. */
int mog_gemm_f32_x3_tn(const float* A, const float* B, float* C, float* colsum, int M, int N,
                       int K, int lda, int ldb, int ldc, int splitk, float* work, long work_elems,
                       void* stream);

/* The same product from operands split beforehand: mog_split3_bf16 writes the
 * three exact bf16 pieces of an fp32 [rows][cols] matrix (piece p at dst + p *
 * piece_stride elements, row pitch ld_dst, columns cols..ld_dst-1 zero);
 * mog_gemm_x3p_tn reads piece p of A at A3 + p * sa and of B at B3 + p * sb
 * (bf16 elements; lda, ldb, sa, sb multiples of 8, 16-byte aligned).
 * npieces = 1: A3 / B3 are plain bf16 operands and the one product is taken
 * (the bf16 configuration's weight gradient of the LSTM kernel's x rows). */
int mog_split3_bf16(const float* src, int rows, int cols, int ld_src, void* dst, int ld_dst,
                    long piece_stride, void* stream);
/* The pieces of a SUM of nsum <= 8 fp32 matrices src + j * sum_stride, added
 * from the last to the first from +0 (the reversed LSTM loop's order of the
 * gate-gradient step sum dGsum, bit for bit): the x-rows gradient's B operand
 * straight from every step's dG, without the running sum in HBM. */
int mog_split3_sum_bf16(const float* src, int nsum, long sum_stride, int rows, int cols,
                        int ld_src, void* dst, int ld_dst, long piece_stride, void* stream);
int mog_gemm_x3p_tn(const void* A3, long sa, const void* B3, long sb, float* C, float* colsum,
                    int M, int N, int K, int lda, int ldb, int ldc, int splitk, int npieces,
                    float* work, long work_elems, void* stream);

/* Build provenance: copies the library's source hash (16 hex digits: sha256
 * of csrc/*.hip, csrc/*.h, include/*.h in sorted order) and a NUL into out
 * (cap >= 17).  The Python host refuses a library whose hash differs from
 * the sources beside it (mog_air/_lib.py). */
int mog_build_id(char* out, int cap);

/* Grouped fp32 weight gradients (mog-asr_amd/csrc/gemm_group.hip): for every
 * problem p of `table` (HOST memory, 10 int64 per problem: A, B, C, colsum
 * device pointers -- colsum may be 0 -- then M, N, K, lda, ldb, ldc),
 * C_p[m][n] += sum_k A_p[k*lda+m] B_p[k*ldb+n] and colsum_p[n] += sum_k
 * B_p[k*ldb+n], as one launch per 24 problems (the problems travel in the
 * kernel argument: graph-capturable with no table upload).  One writer per
 * output element (deterministic): no two problems may share an output.  The
 * weight gradients of the small-batch train step (TF MatMul gradients of
 * vae.py:18-46, the heads of air_model.py:458-520 and the LSTM kernel of
 * :454-456, K = the batch rows). */
int mog_gemm_f32_wgrad_group(const long long* table, int nprob, void* stream);

/* Grouped tall-K weight gradients on bf16 operands (the bf16 configuration's
 * VAE weight / bias gradients, the MatMul / BiasAdd gradients of
 * vae.py:18-46 over all T*B rows): for each problem i < nprob <= 8,
 * out_i[M][N] (ldc) += X_i^T dY_i over K rows and colsum_i[N] += the column
 * sums of dY_i (colsum or colsum[i] may be NULL), X_i [K][lda], dY_i [K][ldb]
 * bf16, 16-byte aligned, lda / ldb multiples of 8, K x ld elements readable.
 * dims: (M, N, lda, ldb, ldc) per problem.  The K rows are cut into nsplit
 * splits whose partial tiles go to `work` (>= mog_wgrad_tn_work_elems floats)
 * and are added in split order by a second launch: deterministic. */
long mog_wgrad_tn_work_elems(int nprob, const int* dims, int nsplit);
int mog_wgrad_tn_bf16(int nprob, const void* const* X, const void* const* dY, float* const* out,
                      float* const* colsum, const int* dims, int K, int nsplit, float* work,
                      long work_elems, void* stream);
/* The same grouped weight gradients on fp32 operands at fp32-level accuracy
 * (the fp32 configuration's VAE weight / bias gradients): X_i, dY_i fp32,
 * 16-byte aligned, lda / ldb even; exact three-piece bf16 splits
 * inside the kernel, six MFMA products per block (as mog_gemm_f32_x3_tn);
 * deterministic. */
int mog_wgrad_tn_x3(int nprob, const float* const* X, const float* const* dY, float* const* out,
                    float* const* colsum, const int* dims, int K, int nsplit, float* work,
                    long work_elems, void* stream);

/* dX = epi(dY W^T) at fp32-level accuracy on the bf16 matrix cores (the VAE
 * input gradients; replaces the MatMul gradients of vae.py:18-46's dense
 * layers w.r.t. their inputs): C[M][N] = sum_k A[m][k] B[n][k], A fp32 [M][lda]
 * split into three bf16 pieces inside the kernel, B = W [N][K] given as the
 * three pieces of mog_split3_bf16 (piece p at B3 + p * sb, row pitch ldb).
 * epi 0: store; 1: C = v * (1 - exp(-aux[m][n])) (dX through softplus; aux =
 * the softplus output, sigmoid(x) = 1 - exp(-softplus(x))).
 * K, ldb, sb multiples of 8; N, lda, ldc, ldaux multiples of 4; deterministic. */
int mog_gemm_x3_nt(const float* A, const void* B3, long sb, float* C, const float* aux, int M,
                   int N, int K, int lda, int ldb, int ldc, int ldaux, int epi, void* stream);

/* C = sigmoid((A B + bias) + scale * eps) for A [M][K] (lda), B [K][N] (ldb):
 * the VAE output layer (vae.py:44-46) with the likelihood noise eps generated
 * in the epilogue -- element (m, n) is lane n % 4 of Philox4x32-10 quad
 * offset + m * N / 4 + n / 4, bit-identical to mog_rng_fill(seed, offset) of
 * an [M][N] buffer read as the aux operand of epi 3.  N % 4 == 0.  Replaces
 * TF's random_normal + add + sigmoid of the decoder (air_model.py:548-550). */
int mog_gemm_f32_sigmoid_philox(const float* A, const float* B, float* C, const float* bias,
                                int M, int N, int K, int lda, int ldb, int ldc, float scale,
                                unsigned long long seed, unsigned long long offset,
                                void* stream);
/* C = epi(sum_s A_s op(B_s)) as one k-ordered chain over K = nseg * kseg
 * (nseg <= 8, kseg % 16 == 0; segment s from A[s] / B[s]); epi 0 or 5.  The
 * five heads' hidden-state gradient dh = sum_z dhid_z W1_z^T in one launch. */
int mog_gemm_f32_kseg(int nseg, const float* const* A, const float* const* B, float* C,
                      const float* bias, const float* Cin, int M, int N, int kseg, int lda,
                      int ldb, int ldc, int transA, int transB, int epi, void* stream);
/* nprob <= 4 independent k-segment chains of one shape (M x N, kseg, lda /
 * ldb / ldc, NT when transB) in ONE launch: C[z] = Cin[z] (or 0) + sum of
 * problem z's nseg[z] segments A_s op(B_s), the problems' segments back to
 * back in the HOST arrays A / B (at most 8 in all); C / Cin / nseg HOST
 * arrays of nprob.  Same chains and bits as nprob mog_gemm_f32_kseg calls.
 * Replaces one AIR-ASR loop step's three head-gradient GEMMs (dh_t, dhg_t,
 * dhg_{t-1} through the z_pres prior; air_model_pr.py's heads). */
int mog_gemm_f32_kseg_group(int nprob, const int* nseg, const float* const* A,
                            const float* const* B, float* const* C, const float* const* Cin, int M,
                            int N, int kseg, int lda, int ldb, int ldc, int transB, void* stream);

/* ---- spatial transformer -------------------------------------------------
 * air/transformer.py:18-175 transformer(U, theta, out_size) for N images:
 * U [N, Hin*Win], theta [N, 6] (row-major 2x3), out [N, Hout*Wout].
 * mode 0: out (fp32) = w;  mode 2: out (bf16) = w;
 * mode 1 fuses the canvas update of air_model.py:665-675 into fp32 out:
 * out[n] += mask[n] != 0 ? z[n] * w : 0 (z, mask [N]). */
int mog_stn_forward(const float* U, int N, int Hin, int Win, const float* theta, int Hout,
                    int Wout, void* out, const float* z, const float* mask, int mode,
                    void* stream);
/* The same with image n reading U[n % u_period] (u_period > 0; 0: U[n]):
 * every loop step's glimpse read of AIR's shared input canvas in one launch
 * (N = T * B, u_period = B). */
int mog_stn_forward_periodic(const float* U, int u_period, int N, int Hin, int Win,
                             const float* theta, int Hout, int Wout, void* out, const float* z,
                             const float* mask, int mode, void* stream);
/* STN write of N images into per-image canvas parts (mode-1 semantics without
 * the read-modify-write): parts[n] = mask[n] ? z[n] * STN(U[n], theta[n]) : 0,
 * stored only on the rows part_rows[n] = lo | hi << 16 (even bounds; rows
 * outside are exactly +0 for axis-aligned theta; all rows otherwise; 0 for an
 * inactive image).  mog_recon_loss sums T such part sets in step order
 * (air_model.py:580-588, 665-675), bit-identical to accumulating. */
int mog_stn_write_parts(const float* U, int N, int Hin, int Win, const float* theta, int Hout,
                        int Wout, const float* z, const float* mask, float* parts,
                        int* part_rows, void* stream);

/* Gradient of transformer() (TF GatherV2 grad = UnsortedSegmentSum + the
 * affine-grid chain): G [N, Hout*Wout] upstream, scaled per image by gscale[n]
 * (may be NULL).  Writes dU [N, Hin*Win] (may be NULL), dtheta [N, 6] (may be
 * NULL) and dot[n] = sum_p G[n,p] * out[n,p] (may be NULL).  u_period /
 * g_period > 0: image n reads U / G row n % period (all loop steps of a batch
 * in one launch against the shared canvas input or canvas gradient). */
int mog_stn_backward(const float* U, int N, int Hin, int Win, const float* theta, int Hout,
                     int Wout, const float* G, const float* gscale, float* dU, float* dtheta,
                     float* dot, int u_period, int g_period, void* stream);
/* The same with the glimpse gradient taken through the VAE output sigmoid
 * (vae.py:44-46, TF SigmoidGrad): dm[n] = bf16((dU[n] * U[n]) * (1 - U[n])), U
 * being the sigmoid output r, written instead of dU (u_period must be 0). */
int mog_stn_backward_sigmoid_bf16(const float* U, int N, int Hin, int Win, const float* theta,
                                  int Hout, int Wout, const float* G, const float* gscale,
                                  void* dm, float* dtheta, float* dot, int u_period, int g_period,
                                  void* stream);
/* The same with dm in fp32 (the reference-precision train step). */
int mog_stn_backward_sigmoid_f32(const float* U, int N, int Hin, int Win, const float* theta,
                                 int Hout, int Wout, const float* G, const float* gscale, float* dm,
                                 float* dtheta, float* dot, int u_period, int g_period,
                                 void* stream);

/* ---- LSTM cell (TF-1.12 BasicLSTMCell, air_model.py:454-456,812-815) -----
 * G [B, 4H] gate pre-activations (i,j,f,o) WITHOUT bias when `bias` != NULL. */
int mog_lstm_cell_forward(const float* G, const float* bias, const float* c_prev, float* c_out,
                          float* h_out, int B, int H, void* stream);
int mog_lstm_cell_backward(const float* G, const float* bias, const float* c_prev,
                           const float* c_cur, const float* dh, const float* dc, float* dG,
                           float* dc_prev, float* dGsum, int B, int H, void* stream);
/* The same with dh = dh + parts[0] + ... + parts[nparts-1] (nparts <= 4, each
 * [B, H], part_stride elements apart, added in part order): the hidden-state
 * gradient GEMM dG_{t+1} Wh^T split over K into nparts products that this
 * launch sums -- at the reference's batch of 64 the split cuts that GEMM's
 * serial K = 4H chain per workgroup by nparts, with no reduction launch. */
int mog_lstm_cell_backward_parts(const float* G, const float* bias, const float* c_prev,
                                 const float* c_cur, const float* dh, const float* dh_parts,
                                 int nparts, long part_stride, const float* dc, float* dG,
                                 float* dc_prev, float* dGsum, int B, int H, void* stream);
/* Two independent cells of one batch in one launch (AIR-ASR's inference and
 * generative LSTMCells, asr_model.py's loop): `cells` is a HOST array of
 * 2 x 5 device pointers {G, bias, c_prev, c_out, h_out} (forward) or
 * 2 x 9 {G, bias, c_prev, c_cur, dh, dc, dG, dc_prev, dGsum} (backward),
 * each cell's NULLs as in the single-cell calls; results bit-identical to two
 * single-cell calls.  Replaces the two rnn_cell calls per step of
 * air/air_model_pr.py's ASR loop. */
int mog_lstm_cell_forward_pair(const float* const* cells, int B, int H, void* stream);
int mog_lstm_cell_backward_pair(const float* const* cells, int B, int H, void* stream);

/* ---- per-step scalars ----------------------------------------------------
 * air_model.py:458-520 (head outputs, scale/shift sampling, theta),
 * :552-577 (theta^-1), :590-663 (concrete z_pres, KL, stop/digits),
 * :677-705 (scale/shift KLs), loop predicate :428-432 via live[step+1].
 * hid/w2/b2: HOST arrays of 5 device pointers (scale-mean, scale-logvar,
 * shift-mean, shift-logvar, z_pres log-odds). rec: [17, B] saved records
 * (slot 16: the z_pres KL term this step added to runloss, for mog_air_runloss).
 * prior_lo_dev (may be NULL): device float read instead of prior_lo -- the
 * annealed z_pres prior (air_model.py:164-184) of a graph-captured train step,
 * whose kernel arguments are fixed at capture. */
int mog_air_step_forward(int B, int HS, int HZ, int step, int train, int use_num_prior,
                         float thr, float temperature, float prior_lo, float prior_bias,
                         float s_pm, float s_pv, float s_plv, float h_pm, float h_pv, float h_plv,
                         const float* const* hid, const float* const* w2,
                         const float* const* b2, const float* eps_scale,
                         const float* eps_shift, const float* u, float* stop, float* runloss,
                         int* digits, int* live, float* rec, float* theta_fwd,
                         float* theta_back, float* scale_out, float* shift_out,
                         float* zprob_out, float* zkl_out, float* skl_out, float* shkl_out,
                         float* zmask, float* zval, float* zc, const float* prior_lo_dev,
                         void* stream);
/* Every loop step in ONE launch (AIR, air_model.py:435-736 with the LSTM
 * chain run first: the heads read h_t only, the step's VAE never feeds the
 * recurrence): steps <= 8; every per-step operand over steps * B rows back to
 * back (step t at the pointer + t * B * width; rec [steps][17][B]; hid head z
 * step t at hid[z] + t * hid_step); prior_bias: HOST array of `steps` values
 * (the per-step marginal bias, air_model.py:600-620).  Writes the bits of
 * `steps` mog_air_step_forward calls except what depends on the batch-wide
 * loop predicate: runloss is not written, rec's z_pres-term slot holds the
 * term the step adds IF it is live, and mog_air_runloss(..., live) applies
 * live[] (set here, reduced over ranks in between under data parallelism). */
int mog_air_step_forward_steps(int steps, int B, int HS, int HZ, int train, int use_num_prior,
                               float thr, float temperature, float prior_lo,
                               const float* prior_bias, float s_pm, float s_pv, float s_plv,
                               float h_pm, float h_pv, float h_plv, const float* const* hid,
                               long hid_step, const float* const* w2, const float* const* b2,
                               const float* eps_scale, const float* eps_shift, const float* u,
                               float* stop, int* digits, int* live, float* rec,
                               float* theta_fwd, float* theta_back, float* scale_out,
                               float* shift_out, float* zprob_out, float* zkl_out,
                               float* skl_out, float* shkl_out, float* zmask, float* zval,
                               float* zc, const float* prior_lo_dev, void* stream);
/* Backward of the above: writes dout [5][B, 2] and dhid [5][B, HS] (head
 * strides dout_hs / dhid_hs elements; dhid_hs == HS means the heads side by
 * side, [B][5][HS] with rows 5 HS apart).  The KL terms this step added to the
 * running loss are weighted by dloss[b] (the loss's cotangent per image), or by
 * the scalar grad_scale when dloss is NULL (a batch-mean loss: 1 / B). */
int mog_air_step_backward(int B, int HS, int train, int use_num_prior, float temperature,
                          float prior_lo, float prior_bias, float s_pm, float s_pv, float h_pm,
                          float h_pv, float grad_scale, const float* dloss, const float* rec,
                          const float* eps_scale,
                          const float* eps_shift, const float* dtheta_fwd,
                          const float* dtheta_back, const float* dot, const float* const* hid,
                          const float* const* w2, float* dout, long dout_hs, float* dhid,
                          long dhid_hs, const float* prior_lo_dev, void* stream);
/* The same over `steps` loop steps in one launch (AIR's reversed loop: every
 * input of a step's head backward is final before the loop -- the STN
 * backwards run over all T*B rows first): rows b = t * B + i, the records of
 * step t at rec + t * 17 * B ([T][17][B], as the forward writes them), dloss
 * per image i, every other operand over the steps * B rows back to back.
 * prior_bias is one value for all steps (no per-step marginal).  Bits of
 * `steps` single-step calls. */
int mog_air_step_backward_steps(int steps, int B, int HS, int train, int use_num_prior,
                                float temperature, float prior_lo, float prior_bias, float s_pm,
                                float s_pv, float h_pm, float h_pv, float grad_scale,
                                const float* dloss, const float* rec, const float* eps_scale,
                                const float* eps_shift, const float* dtheta_fwd,
                                const float* dtheta_back, const float* dot,
                                const float* const* hid, const float* const* w2, float* dout,
                                long dout_hs, float* dhid, long dhid_hs, const float* prior_lo_dev,
                                void* stream);

/* ---- VAE latent sample + KL (air/vae.py:27-30, air_model.py:718-736) ----
 * z_bf16 (may be NULL): bf16 copy of z with row stride ld_zb (GEMM operand).
 * runloss may be NULL (vkl only; mog_air_runloss adds it later). */
int mog_vae_sample_forward(int B, int Z, float v_pm, float v_pv, float v_plv, const float* mu,
                           const float* lv, const float* eps, float* z, void* z_bf16, int ld_zb,
                           const float* act, float* runloss, float* vkl, void* stream);
/* Per-image running loss of T steps replayed from the records in the order the
 * loop accumulates it (air_model.py:622-736: per step the z_pres term, then,
 * for an active image, scale KL, shift KL, VAE KL), starting from +0:
 * bit-identical to accumulating step by step.  rec: [T][rec_step_stride]
 * (mog_air_step_forward records), skl/shkl/vkl: [T, B].  Lets the VAE of all
 * T steps run after the recurrent loop as one set of launches over T*B rows
 * (AIR: the VAE output never feeds the recurrence).  live (may be NULL): the
 * loop-predicate flags [T+1] of mog_air_step_forward_steps, applied first: the
 * z_pres term of a step that is not live becomes 0 and rec's z_pres-term and
 * live slots are rewritten to what T single-step launches record. */
int mog_air_runloss(int T, int B, float* rec, long rec_step_stride, const float* skl,
                    const float* shkl, const float* vkl, float* runloss, const int* live,
                    void* stream);
/* ---- fused per-object step, bf16 configuration ----
 * One launch per loop step: glimpse = STN(x, theta_f) (transformer.py:18-175),
 * the glimpse VAE (vae.py:5-48: recognition 784->512->256 softplus, mean /
 * log-variance 256->50, z = mu + eps*sqrt(exp(lv)), generative 50->256->512
 * softplus, r = sigmoid(512->784 + std*eps_x)), the VAE KL into runloss under
 * `mask` (air_model.py:718-736), and this step's canvas contribution
 * canvas_part = mask ? zval * STN(r, theta_b) : 0 (air_model.py:580-588,
 * 665-675; summed in step order by mog_recon_loss).  Only the rows that can be
 * nonzero are stored: part_rows[b] = lo | hi << 16 records the stored row range
 * [lo, hi) of image b (0 for an inactive image); every other pixel is +0.
 * wt[7] are the bf16 W^T packs in B-fragment order (mog_cvt_bf16_batch
 * transpose 2) in the order recognition_1, recognition_2, rec_mean, rec_log_variance,
 * generative_1, generative_2, gen_mean; bias[7] fp32 likewise.  eps_x: read
 * from `eps_x` [B,784] when eps_gen == 0; otherwise generated in-kernel as the
 * Philox normals mog_rng_fill(eps_x, B*784, eps_seed, eps_offset, 1) would
 * have written (bit-identical; eps_x may then be NULL).  Saved for the
 * backward: gb/a1b/a2b/zb/d1b/d2b (bf16, zb row stride 56), mu/lv/z (fp32) --
 * a1b/a2b/zb/d1b/d2b/mu/lv NULL for a forward-only step (evaluation /
 * inference; z, the reported latents, is written when given); r (fp32) is
 * always written; in the forward-only form gb is not written either (it may
 * be NULL).  Workgroups of 64 images (32 below B = 16,384),
 * every phase of a tile in sequence on the whole CU.
 * Shapes must be the reference defaults (W 28, 512/256, Z 50, 256/512):
 * anything else returns MOG_ERR_INVALID.  Replaces the per-step sequence
 * air_model.py:523-588 (stn_forward + 6 GEMMs + vae_sample + stn accumulate).
 * x_period > 0 (all T steps in one launch: B = T * x_period rows, row b reads
 * image x[b % x_period]) requires x_period % 64 == 0 and runloss == NULL;
 * x_period <= 0 means B. */
int mog_stn_vae_step_forward(int B, int C, int W, int R1, int R2, int Z, int G1, int G2,
                             const float* x, const float* theta_f, const float* theta_b,
                             const float* mask, const float* zval, const float* eps_z,
                             const float* eps_x, int eps_gen, unsigned long long eps_seed,
                             unsigned long long eps_offset, const void* const* wt,
                             const float* const* bias, float lik_std, float v_pm, float v_pv,
                             float v_plv, float* canvas_part, int* part_rows, float* runloss,
                             float* vkl, void* gb,
                             void* a1b, void* a2b, float* mu, float* lv, float* z, void* zb,
                             void* d1b, void* d2b, float* r, int x_period, void* stream);

/* fp32 MFMA B-fragment packs of n <= 8 weight matrices W[i] [K[i]][N[i]]
 * (row-major fp32, TF [in, out]) into out[i] ((K+15)/16 * (N+15)/16 KiB):
 * fragment (ks, ct) at ((ks * NCT + ct) * 64 + lane) * 4 floats holds
 * W[16 ks + 4 kk + g][16 ct + li], kk < 4, lane = 16 g + li; zero outside W.
 * The weight operand of mog_stn_vae_step_forward_f32. */
int mog_pack_frag_f32(int n, const float* const* W, const int* K, const int* N,
                      float* const* out, void* stream);

/* The fp32 fused step: mog_stn_vae_step_forward at the reference precision,
 * bit-identical to the unfused fp32 sequence (mog_stn_forward, the seven
 * mog_gemm_f32 layers with their pre-activations, mog_vae_sample_forward,
 * mog_gemm_f32_sigmoid_philox / EPI_SIGMOID_NOISE, mog_stn_write_parts).
 * wt[7]: mog_pack_frag_f32 packs of the seven VAE weights (order as
 * mog_stn_vae_step_forward's), bias[7] fp32.  Saved for the backward, fp32:
 * g [B,784], a1 [B,512], a2 [B,256], mu/lv [B,50], d1 [B,256], d2 [B,512]
 * -- all given, or all NULL (forward only); the pre-activations a1pre, a2pre,
 * d1pre, d2pre are optional (NULL: not stored; the softplus backward needs
 * only the outputs, epi 4 of mog_gemm_f32 / 1 of mog_gemm_x3_nt); z
 * [B,50] and r [B,784] are always written.  Tiles of 32 images: x_period > 0
 * requires x_period % 32 == 0 and runloss == NULL.  Reference VAE shape only.
 * Replaces air_model.py:523-588 at fp32. */
int mog_stn_vae_step_forward_f32(int B, int C, const float* x, const float* theta_f,
                                 const float* theta_b, const float* mask, const float* zval,
                                 const float* eps_z, const float* eps_x, int eps_gen,
                                 unsigned long long eps_seed, unsigned long long eps_offset,
                                 const float* const* wt, const float* const* bias, float lik_std,
                                 float v_pm, float v_pv, float v_plv, float* canvas_part,
                                 int* part_rows, float* runloss, float* vkl, float* g,
                                 float* a1pre, float* a1, float* a2pre, float* a2, float* mu,
                                 float* lv, float* z, float* d1pre, float* d1, float* d2pre,
                                 float* d2, float* r, int x_period, void* stream);

/* dmu/dlv fp32 [B,Z] and/or bf16 copies with row stride ld_b (any may be NULL,
 * but one complete pair must be given). */
int mog_vae_sample_backward(int B, int Z, float v_pm, float v_pv, float grad_scale,
                            const float* mu, const float* lv, const float* eps, const float* dz,
                            const float* act, float* dmu, float* dlv, void* dmu_bf16,
                            void* dlv_bf16, int ld_b, void* stream);
/* TF SigmoidGrad: dm = dr * r * (1 - r) (vae.py:46); dm fp32 or bf16. */
int mog_sigmoid_backward(const float* r, const float* dr, void* dm, long n, int out_bf16,
                         void* stream);

/* ---- bf16-operand GEMM (configs[1]: bf16 glimpse-VAE) --------------------
 * tn = 0: C[m][n] = sum_k A[m*lda+k] B[n*ldb+k]   (forward with W^T packed,
 *         dX with W packed);  K % 8 == 0 (zero-padded buffers).
 * tn = 1: C[m][n] = sum_k A[k*lda+m] B[k*ldb+n]   (dW = X^T dY, split-K,
 *         epi 4 fp32 atomics, colsum = fused bias gradient).
 * epi: 0 store(+bias) 1 softplus 2 sigmoid(acc+bias+aux*aux_scale) [aux fp32]
 *      3 acc*(1-exp(-aux)) [aux = softplus output, bf16] 4 atomic-add.
 * A, B, aux(epi 3): bf16; C bf16 when out_bf16 else fp32; Cin fp32 (ldc). */
int mog_gemm_bf16(int batch, const void* const* A, const void* const* B, void* const* C,
                  const float* const* bias, const float* const* Cin, const void* const* aux,
                  float* const* colsum, int M, int N, int K, int lda, int ldb, int ldc,
                  int ldaux, int tn, int epi, int out_bf16, float aux_scale, int splitk,
                  void* stream);
/* fp32 -> bf16 weight packing: dst[r][c] = src[c][r] (transpose) or src[r][c],
 * zero outside the (src_rows, src_cols) source extent. */
int mog_cvt_bf16(const float* src, int src_rows, int src_cols, int ld_src, void* dst, int rows,
                 int cols, int ld_dst, int transpose, void* stream);
/* Up to 16 of the above in one launch; dims[7*j ..] = src_rows, src_cols,
 * ld_src, rows, cols, ld_dst, transpose of job j.  transpose == 2 packs W^T
 * (W = src [src_rows = in][src_cols = out]) in MFMA B-fragment order for
 * mog_stn_vae_step_forward: rows = out padded to 16, cols = in padded to 32,
 * element ((ct*(cols/32) + ks)*64 + lane)*8 + q = W[ks*32 + 8*(lane/16) + q]
 * [ct*16 + lane%16], zero outside the source (ld_dst unused). */
int mog_cvt_bf16_batch(int njobs, const float* const* src, void* const* dst, const int* dims,
                       void* stream);

/* ---- reconstruction loss (air_model.py:866-900) -------------------------- */
/* With nparts == 0 the canvas [B, C2] is read.  With nparts > 0 it is the
 * step-ordered sum of the per-step contributions parts[t] (stride part_stride
 * elements; written by mog_stn_vae_step_forward) and is stored to `canvas`
 * when that is non-NULL.  part_rows (may be NULL: parts fully stored) [nparts,
 * B]: rows [lo, hi) = (v & 0xffff, v >> 16) of part t / image b that were
 * stored, the part being +0 elsewhere (C = canvas side, C*C == C2). */
int mog_recon_loss(const float* x, float* canvas, const float* parts, int nparts,
                   long part_stride, const int* part_rows, int C, const float* runloss, const int* digits,
                   const int* targets, int B, int C2, float grad_scale, float* recon,
                   float* bce, float* mse, float* loss, float* acc, float* dcanvas,
                   void* stream);
/* out[k] = mean_b a_k[b] for the non-NULL a_k (k < 4). */
int mog_batch_mean(const float* a0, const float* a1, const float* a2, const float* a3, int B,
                   float* out, void* stream);
/* out[n] += sum_r X[r*ld + n]  (BiasAddGrad) */
int mog_colsum_add(const float* X, int R, int N, int ld, float* out, void* stream);
/* Weight and bias gradients of the heads' 1- / 2-column output layers
 * (air_model.py:462-499 backward): gw[z] [HS, k[z]] += hid[z]^T dout[z],
 * gb[z] [k[z]] += column sums of dout[z] (gb may be NULL), over R rows; hid[z]
 * [R, HS], dout[z] [R, 2] (the unused column of a 1-column head ignored).
 * Deterministic: 128-row chunks summed in row order into `work`, the chunks
 * added in chunk order by a second launch.  nheads <= 5, HS < 128;
 * work_elems >= mog_heads_output_wgrad_work_elems(nheads, R, HS). */
long mog_heads_output_wgrad_work_elems(int nheads, int R, int HS);
int mog_heads_output_wgrad(int nheads, const float* const* hid, const float* const* dout,
                           float* const* gw, float* const* gb, const int* k, int R, int HS,
                           float* work, long work_elems, void* stream);
int mog_add(const float* a, const float* b, float* out, long n, void* stream);

/* ---- optimizer (air_model.py:941-999) ------------------------------------
 * Per-tensor inf/nan -> 0, clip_by_norm(clip), TF ApplyAdam with lr_t given.
 * off/len: tensor table; block_tensor/block_start: block -> (tensor, first
 * element), chunks of mog_optim_chunk_elems() elements; all device arrays.
 * params / grads / m / v 16-byte aligned, every off[] a multiple of 4.
 * sumsq: device scratch of nblocks floats (each chunk's sum of squares; a
 * tensor's norm is summed from them in chunk order: deterministic, no
 * atomics); sumsq == NULL skips the NaN/Inf zeroing and the clip
 * (gradient_clipping_norm=None, air_model.py:948). */
int mog_optim_chunk_elems(void);
int mog_clip_adam(float* params, float* grads, float* m, float* v, const long* off,
                  const long* len, const int* block_tensor, const long* block_start,
                  int nblocks, float* sumsq, float clip, float lr_t, float beta1, float beta2,
                  float eps, void* stream);

/* ---- generation loop prior draws (air_model.py:1001-1146, vae.py:51-86) --
 * Per image i < G: s = sigmoid(s_pm + eps_scale[i] sqrt(exp(s_plv))),
 * (tx, ty) = tanh(h_pm + eps_shift[i][:] sqrt(exp(h_plv))), theta_back[i] =
 * [[1/s, 0, -tx/s], [0, 1/s, -ty/s]]; per latent element z = v_pm + eps_z
 * sqrt(exp(v_plv)).  Replaces the scale / shift / rec_sample scopes of
 * _create_generation (:1013-1035) and vae_generation (vae.py:63-66). */
int mog_generation_prior(int G, int Z, float s_pm, float s_plv, float h_pm, float h_plv,
                         float v_pm, float v_plv, const float* eps_scale, const float* eps_shift,
                         const float* eps_z, float* theta_back, float* scale, float* shift,
                         float* z, void* stream);

/* ---- AIR-ASR cells and structural losses (air_number_bbox_location.py) ----
 * Record layout rec[step][28][B]: sm0 sm1 slv0 slv1 sl0 sl1 cm clv cl s tx ty
 * gsm0 gsm1 gslv0 gslv1 plo lo y z act_old act live zkl skl shkl prn zprob
 * (zkl / skl / shkl masked as the reference's tf.where, prn live-gated).
 * w[20] (TF [in,out] layout): inf_shift dense_1 W,b, dense_3 W,b; inf_scale
 * dense W,b [258,64], dense_1 W,b [66,1], dense_2 W,b, dense_3 W,b; gen_shift
 * dense_1 W,b, dense_3 W,b; z_pres prior dense_1 W,b; z_pres log-odds
 * dense_1 W,b.  hid[8] [B,64]: post-relu hidden of inf_shift m / v, z_pres
 * log-odds, gen_shift m / v, z_pres prior (null with fix_steps >= 0), and the
 * inf_scale m / v chains over h (finished in place: + shift latent terms,
 * bias, relu).  gammas[8] = num, margin, element, bbox, size, area, area_min,
 * area_max.  T <= 8 steps, <= 8 allowed counts. */
/* U rows [z (Z) | ss (3) | h (H) | 0] of the two LSTMCell inputs (:403-412,
 * :457-463); null sources read as zeros.  out2 != NULL: the second cell's rows
 * [z | ss | h2 | 0] into out2 in the same launch. */
int mog_asr_pack(int B, int Z, int H, int ld, const float* z, const float* ss, const float* h,
                 float* out, const float* h2, float* out2, void* stream);
/* dz = dU[:, :Z] + dUg[:, :Z] (acc_dz: dz += that sum, the carry added into
 * an existing latent gradient); dss likewise (stored); dh += dU[:, Z+3:];
 * dhg += dUg[:, Z+3:] */
int mog_asr_unpack(int B, int Z, int H, int ld, const float* dU, const float* dUg, float* dz,
                   float* dss, float* dh, float* dhg, int acc_dz, void* stream);
/* The same with dU / dUg given as nparts <= 4 K parts of their GEMM (part j at
 * + j * part_stride elements), summed in part order (the small-batch recurrent
 * input gradient split over K = 4H, as mog_lstm_cell_backward_parts). */
int mog_asr_unpack_parts(int B, int Z, int H, int ld, const float* dU, const float* dUg,
                         int nparts, long part_stride, float* dz, float* dss, float* dh,
                         float* dhg, int acc_dz, void* stream);
/* heads, latents, theta, concrete z_pres, KLs, entropy, stop / counts /
 * live flag of one step (:414-772) */
int mog_asr_step_forward(int B, int step, int train, int fix_steps, float thr, float temperature,
                         float scale_prior_mean, float scale_prior_var, float scale_prior_logvar,
                         float gamma_num, const float* const* w, float* const* hid,
                         const float* eps_shift, const float* eps_scale, const float* u,
                         float* stop, int* digits, int* live, float* rec, float* theta_fwd,
                         float* theta_back, float* ss, float* scale, float* shift, float* zprob,
                         float* zmask, float* zval, float* zc, void* stream);
/* per image KL sums (klsum, the reconstruction kernel's runloss), pr_loss
 * and its area / out / size / overlap terms over the executed steps; zsum[t]
 * = sum_b z_pres_prob (to be all-reduced over ranks for the margin loss)
 * (:917-935, :1017-1069).  rec [T][28][B], vkl / zmask [T][B]. */
int mog_asr_terms(int B, int T, int C, int nc, const int* cons, const float* gammas,
                  const float* rec, const float* vkl, const float* zmask, const int* live,
                  float* klsum, float* pr, float* area, float* out, float* size, float* overlap,
                  float* zsum, void* stream);
/* loss[b] = (loss[b] + pr[b]) + element[b]; margin[0] (:970-1015, :1078-1079);
 * cons / gammas are HOST arrays */
int mog_asr_finalize(int B, int T, int C, int nc, const int* cons, const float* gammas,
                     float inv_batch_global, const float* rec, const int* live, const float* zsum,
                     const float* pr, float* loss, float* element, float* margin, void* stream);
/* dreg [T][4][B]: d loss / d (s, tx, ty, lo) from the regularisers */
int mog_asr_terms_backward(int B, int T, int C, int nc, const int* cons, const float* gammas,
                           float grad_scale, float inv_batch_global, const float* rec,
                           const int* live, const float* zsum, float* dreg, void* stream);
/* one step's backward of mog_asr_step_forward: douts [B][12] = d(sm0 sm1 slv0
 * slv1 lo gsm0 gsm1 gslv0 gslv1 plo cm clv), dpre[8] [B,64] hidden-layer
 * pre-activation gradients; dss [B,3] = gradient reaching this step's latents
 * from the next step's LSTM inputs (or null) */
int mog_asr_step_backward(int B, int train, int fix_steps, float temperature,
                          float scale_prior_mean, float scale_prior_var, float grad_scale,
                          const float* const* w, float* const* hid, const float* rec,
                          const float* eps_shift, const float* eps_scale, const float* dtheta_fwd,
                          const float* dtheta_back, const float* dot, const float* dreg,
                          const float* dss, float* douts, float* const* dpre, void* stream);

/* ---- noise (tf.random_normal / random_uniform sites, perf mode) --------- */
int mog_rng_fill(float* out, long n, unsigned long long seed, unsigned long long offset,
                 int normal, void* stream);
/* Up to 8 buffers in one launch (host arrays): buffer j is bit-identical to
 * mog_rng_fill(out[j], n[j], seed, offset[j], normal[j]).  The step's five
 * noise draws (air_model.py:191, vae.py:29,44, concrete.py:23). */
int mog_rng_fill_batch(int nbuf, float* const* out, const long* n, unsigned long long seed,
                       const unsigned long long* offset, const int* normal, void* stream);

/* ---- step resets ----------------------------------------------------------
 * Up to 8 buffers of n[j] 32-bit words set to value[j] in one launch (host
 * arrays): the loop state at the start of a step (tf.while_loop's initial
 * values, air_model.py:815-826) and the zeroed gradient accumulators. */
int mog_fill32_batch(int nbuf, void* const* dst, const long* n, const unsigned* value,
                     void* stream);
/* Up to 8 copies of n[j] 32-bit words src[j] -> dst[j] in one launch (a
 * captured step's inputs into the graph's static buffers). */
int mog_copy32_batch(int nbuf, void* const* dst, const void* const* src, const long* n,
                     void* stream);
/* Up to 8 fp32 transposes in one launch: dst[j] [cols][rows] = src[j] [rows][cols]
 * (the small-batch forward's W^T copies of the VAE layers whose N or K is the
 * 50-wide latent: NT GEMM forms with the same k-ordered chains). */
int mog_transpose32_batch(int nbuf, float* const* dst, const float* const* src, const int* rows,
                          const int* cols, void* stream);

/* ---- measurement instrument (no reference counterpart) -------------------
 * dst[i] = src[i] for n4 float4s (16-byte aligned): the copy bandwidth the
 * bench quotes beside the HBM spec.  (The test-only instruments mog_spin and
 * mog_lds_poison live in libmog_air_test.so, include/mog_air_test.h.) */
int mog_copy_f4(const float* src, float* dst, long n4, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MOG_AIR_H */
