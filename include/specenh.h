/*
 * specenh.h — C-ABI of the MI355X-native spectrogram-enhancement hot path.
 *
 * libspecenh.so (hipcc, gfx950) exports exactly these symbols. Signatures use
 * plain pointers, sizes and a HIP stream handle (void*, may be NULL = default
 * stream); no torch types. Device pointers must be on the current HIP device.
 * Every entry point returns 0 on success or a negative SPECENH_E* code; the text
 * of the last error on the calling thread is available from
 * specenh_last_error().
 *
 * The reference (PlasmaControl/spectrogram-enhancement) has no FFI: its hot path
 * is Python calling scipy/numpy. Each entry point below names the reference
 * call it replaces; the Python host layer (specenh.pipeline_data, specenh.svd)
 * keeps the reference's function names and argument meanings on top of these.
 */
#ifndef SPECENH_H
#define SPECENH_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPECENH_OK 0
#define SPECENH_EINVAL -1     /* bad argument (maps to ValueError at the Python boundary) */
#define SPECENH_EUNSUPPORTED -2 /* valid for scipy, not implemented here (NotImplementedError) */
#define SPECENH_EHIP -3       /* HIP runtime error (RuntimeError) */
#define SPECENH_ENOMEM -4
#define SPECENH_ERANGE -5     /* index out of range, as the reference raises (IndexError) */

/* Output-mode flags for specenh_stft_psd. */
#define SPECENH_STFT_LOG 1          /* natural log(P + eps)                  pipeline_data.py:33 */
#define SPECENH_STFT_NORMALIZE 2    /* per-spectrogram min-max (implies LOG) pipeline_data.py:34 */
#define SPECENH_STFT_DROP_NYQUIST 4 /* drop the last frequency row         pipeline_data.py:35 */
/* One real frame per complex FFT instead of two (no reference counterpart: an accuracy
 * mode). The two-for-one FFT gives a bin at a spectral null the partner frame's fp32
 * rounding; EXACT keeps the reference's 1e-5 on such bins for twice the FFT work. The
 * numpy-compat entries (specgr, specgr_array) set it; the throughput paths do not. */
#define SPECENH_STFT_EXACT 8

/* detrend / scaling codes (the 'detrend' and 'scaling' keys of spec_params,
 * pipeline_data.py:77-84). */
#define SPECENH_DETREND_NONE 0
#define SPECENH_DETREND_CONSTANT 1
#define SPECENH_DETREND_LINEAR 2
#define SPECENH_SCALING_DENSITY 0
#define SPECENH_SCALING_SPECTRUM 1

const char* specenh_last_error(void);
const char* specenh_version(void);

/* Kernel-variant switches (no reference counterpart: A/B tests of kernels that compute
 * the same result). name = "CONV_NO_S2", "PATCH_WSPLIT", ... (an optional "SPECENH_"
 * prefix is accepted). Each is read from the environment variable SPECENH_<name> once per
 * process; afterwards only these calls change it. Unknown names: SPECENH_EINVAL. */
int specenh_set_variant(const char* name, int value);
int specenh_get_variant(const char* name, int* value);

/* Symbol (as the HIP runtime names it, mangled) of the last kernel this host thread
 * launched through the library, "" before the first launch: measurements key their
 * rocprofv3 PMC records by it (bench.py, tools/conv_one.py). */
const char* specenh_last_kernel_name(void);
/* Number of kernels this host thread has launched through the library: the i-th launch is
 * the i-th specenh dispatch of the thread in a rocprofv3 trace (tools/pmc_workload.py). */
long long specenh_launch_count(void);
/* Symbol of this thread's launch number `index` (0-based, as counted by
 * specenh_launch_count) while it is among the thread's last 256 launches, else "". */
const char* specenh_kernel_name_at(long long index);

/* Make stream `waiter` wait for the work enqueued on stream `signaler` so far (both
 * hipStream_t of one device, not necessarily the current one: the event lives on the
 * signaler's device; no reference counterpart: the AE backward's fork and join of its
 * weight-gradient stream). The event is recorded without the system-scope fence
 * (hipEventDisableSystemFence) when `device_scope` is nonzero: both streams are on one
 * device. Events come from a per-device ring (hipEventDisableTiming). */
int specenh_stream_wait(void* waiter, void* signaler, int device_scope);

/* Number of frames T = (length - nperseg) / (nperseg - noverlap) + 1 that
 * scipy.signal.spectrogram produces (no boundary padding), or a negative error. */
long long specenh_stft_frames(long long length, int nperseg, int noverlap);

/* ---------------------------------------------------------------- STFT-PSD
 * A plan holds the device-resident tables (window, twiddles) for one
 * (nperseg, noverlap, window, fs, scaling, detrend, eps) and one device. It
 * replaces the per-call setup inside scipy.signal.spectrogram
 * (scipy/signal/_spectral_py.py:2079-2093: window cast, scale) as called from
 * spec_denoising/pipeline_data.py:32.
 * window_host: nperseg float64 coefficients (already the periodic window).
 * Creating a plan allocates; launching with it does not (graph-capturable). */
typedef struct specenh_stft_plan specenh_stft_plan;

int specenh_stft_plan_create(specenh_stft_plan** plan, int nperseg, int noverlap,
                             const double* window_host, double fs, int scaling, int detrend,
                             double eps);
int specenh_stft_plan_destroy(specenh_stft_plan* plan);

/* Bytes of device workspace specenh_stft_psd needs for `batch` spectrograms. */
size_t specenh_stft_workspace_bytes(const specenh_stft_plan* plan, long long batch);

/* Batched spectrogram of `batch` real fp32 signals.
 * Replaces, per signal, spec_denoising/pipeline_data.py:32-35
 *   f, t, Sxx = scipy.signal.spectrogram(sig_in, nperseg, noverlap, fs, window,
 *                                        scaling, detrend)        (flags = 0)
 *   Sxx = np.log(Sxx + eps)                                        (| LOG)
 *   Sxx = (Sxx - min) / (max - min)                                (| NORMALIZE)
 *   Sxx = Sxx[:-1, :]                                              (| DROP_NYQUIST)
 * x:   device fp32, signal b starts at x + b*x_stride, `length` samples used.
 * out: device fp32 [batch][F][T], F = nperseg/2 + 1 (or nperseg/2 with
 *      DROP_NYQUIST), frequency-major like scipy.
 * workspace: device, >= specenh_stft_workspace_bytes(plan, batch) bytes.
 * nperseg must be a power of two in [64, 4096]. */
int specenh_stft_psd(const specenh_stft_plan* plan, const float* x, long long batch,
                     long long length, long long x_stride, float* out, int flags,
                     void* workspace, void* stream);
/* As specenh_stft_psd with fp16 samples (x: _Float16, x_stride in elements), widened to
 * fp32 on load — the same arithmetic as specenh_stft_psd on x converted to fp32, without
 * the conversion pass (the C5 stream's fp16 shots). nperseg <= 1024; one workgroup per
 * spectrogram (no team schedule, no workspace). */
int specenh_stft_psd_f16(const specenh_stft_plan* plan, const void* x, long long batch,
                         long long length, long long x_stride, float* out, int flags,
                         void* stream);

/* ---------------------------------------------------------------- cross spectrum
 * Per-segment cross-spectral density of signal pairs: the
 * arithmetic behind interferometer/crosspowerspec.py:39 (ae_co2(signal1, signal2, t),
 * whose source co2_deps is absent) restated as scipy's two-signal _spectral_helper
 * (scipy/signal/_spectral_py.py, mode='psd'): per frame detrend, window, rfft of both,
 *   Pxy = conj(X) * Y * scale, one-sided bins 1..N/2-1 doubled,
 * out [batch][F][T] frequency-major, F = nperseg/2 + 1, T = specenh_stft_frames(...).
 * scipy.signal.csd(x, y) is the mean of Pxy over T. x, y: device fp32, pair b at
 * x + b*x_stride, y + b*y_stride. mode COMPLEX writes float2 (re, im); AMPLITUDE writes
 * |Pxy| as float. nperseg: a power of two in [64, 4096]; batch <= 65535 per call. */
#define SPECENH_CSD_COMPLEX 0
#define SPECENH_CSD_AMPLITUDE 1
typedef struct specenh_csd_plan specenh_csd_plan;
int specenh_csd_plan_create(specenh_csd_plan** plan, int nperseg, int noverlap,
                            const double* window_host, double fs, int scaling, int detrend);
int specenh_csd_plan_destroy(specenh_csd_plan* plan);
int specenh_csd(const specenh_csd_plan* plan, const float* x, const float* y, long long batch,
                long long length, long long x_stride, long long y_stride, void* out, int mode,
                void* stream);

/* ---------------------------------------------------------------- SVD denoiser
 * Batched replacement for denoiseSignal(matrix, start, stop, use_optimal=False)
 * (spec_denoising/denoising_by_svd.ipynb:188-229):
 *   u, s, vh = np.linalg.svd(A, full_matrices=False)
 *   out = u[:, start:stop] @ diag(s[start:stop]) @ vh[start:stop, :]
 * with the notebook's clamping (start < 0 -> 0, stop > r -> r, r = min(m, n)) followed by
 * Python slicing: a negative stop counts from the end (stop + r, floored at 0), an empty
 * slice gives zeros. A: device fp32, matrix b at A + b*a_stride, row-major m x n.
 * out: device fp32 [batch][m][n]. Kept ranges reachable through a top-K singular subspace
 * with K <= 40 (K = stop, or start when stop == r) use fp32-MFMA subspace iteration; any
 * other range (wide ranges, the bottom of the spectrum) uses fp64 eigenvectors of the Gram
 * matrix and needs min(m, n) <= 256 (SPECENH_EUNSUPPORTED otherwise).
 * workspace: >= specenh_svd_denoise_workspace_bytes(batch, m, n, start, stop) bytes
 * (specenh_svd_workspace_bytes(batch, m, n, K) is the same for the top-K forms). */
size_t specenh_svd_workspace_bytes(long long batch, int m, int n, int kmax);
size_t specenh_svd_denoise_workspace_bytes(long long batch, int m, int n, int start, int stop);
int specenh_svd_denoise(const float* A, long long batch, int m, int n, long long a_stride,
                        int start, int stop, float* out, void* workspace, void* stream);
/* The same with the output written as out_dtype (SPECENH_DTYPE_F32 / _BF16 / _F16, codes
 * below): the C5 stream hands the denoised spectrograms to the fp16 autoencoder without a
 * separate cast pass. Arithmetic is unchanged (fp32, rounded once at the store). */
int specenh_svd_denoise_ex(const float* A, long long batch, int m, int n, long long a_stride,
                           int start, int stop, void* out, int out_dtype, void* workspace,
                           void* stream);

/* Gavish-Donoho optimal hard-threshold modes of the same denoiser:
 *   num_sing = #{ s_i > omega(beta) * median(s) },  beta = min(m, n) / max(m, n),
 *   omega(beta) = 0.56 beta^3 - 0.95 beta^2 + 1.82 beta + 1.43   (denoising_by_svd.ipynb:155-159)
 *   SPECENH_SVD_OPTIMAL  keep u[:, 0:num_sing-1]: denoiseSignal(A, use_optimal=True)
 *                        (:210-228; num_sing == 1 gives zeros, num_sing == 0 gives stop = -1,
 *                        i.e. components [0, r-1))
 *   SPECENH_SVD_COMPUTE  keep components [1, 2 num_sing): computeSignal(A) (:161-186); when
 *                        2 num_sing > min(m, n) the notebook's s[idx] raises IndexError ->
 *                        SPECENH_ERANGE (out's contents unspecified).
 * The singular values and vectors come from the fp64 Gram matrix (Householder
 * tridiagonalisation, Sturm bisection for the median, the count and each kept eigenvalue,
 * inverse iteration, reflectors applied back), per matrix, with no host round trip for
 * SPECENH_SVD_OPTIMAL (SPECENH_SVD_COMPUTE synchronises `stream` once to raise the
 * IndexError). Needs min(m, n) <= 256. num_sing (device int[batch]) and median_sv (device
 * double[batch]) are optional outputs. */
#define SPECENH_SVD_OPTIMAL 0
#define SPECENH_SVD_COMPUTE 1
size_t specenh_svd_optimal_workspace_bytes(long long batch, int m, int n);
int specenh_svd_denoise_optimal(const float* A, long long batch, int m, int n, long long a_stride,
                                int mode, float* out, int* num_sing, double* median_sv,
                                void* workspace, void* stream);

/* ---------------------------------------------------------------- conv autoencoder
 * Primitives under the Keras-shaped facade (specenh.keras) that replaces the model of
 * VAE/manual_scan_3layers.py:186-212 (Conv2D / MaxPooling2D / Conv2DTranspose,
 * padding "same", Adam + binary_crossentropy). Tensors are NHWC, device resident.
 * dtype codes: SPECENH_DTYPE_F32 / _BF16 / _F16 (MFMA operands and activations;
 * accumulation, biases, master weights, weight gradients and the loss stay fp32). */
#define SPECENH_DTYPE_F32 0
#define SPECENH_DTYPE_BF16 1
#define SPECENH_DTYPE_F16 2
#define SPECENH_DTYPE_F64 3 /* label filters only */
#define SPECENH_ACT_NONE 0
#define SPECENH_ACT_RELU 1
#define SPECENH_ACT_SIGMOID 2

/* Implicit-GEMM convolution: out[m][co] = act(sum_k A[m][k] * w_gemm[co][k] + bias[co]),
 * m = (n, oy, ox) over [N][OH][OW], k = (ky, kx, ci) over [KH][KW][C]; w_gemm is the
 * N-major GEMM operand [CO][KH][KW][C] ("OHWI"),
 * A[m][k] = in[n][iy][ix][ci] with vy = oy*stride - pad_t + ky, iy = vy / in_dil when
 * vy >= 0, vy % in_dil == 0 and iy < IH (else 0); likewise x with pad_l.
 *   Conv2D(k, "same") forward       stride 1, pad (k-1)/2, in_dil 1,
 *                                   w_gemm[co][ky][kx][ci] = kernel[ky][kx][ci][co]
 *   Conv2DTranspose(k, 2, "same")   stride 1, pad k-1-(k-2)/2, in_dil 2,
 *                                   w_gemm[co][ky][kx][ci] = kernel[k-1-ky][k-1-kx][co][ci]
 *   their input gradients           (see specenh_weight_flip_transpose)
 * A dilated input (in_dil 2, stride 1) is computed as in_dil^2 dense output phases; the
 * zero holes are never gathered or multiplied.
 * logits (optional, fp32 [M][CO]) receives the pre-activation; mask (optional, dtype
 * [M][CO]) zeroes outputs where mask <= 0 (backward through a ReLU); out is fp32 when
 * out_f32 != 0, else dtype. bias may be NULL.
 * pool2 != 0 fuses the following MaxPooling2D((2,2)): out is [N][OH/2][OW/2][CO] (dtype)
 * and argmax (optional, same shape, uint8 dy*2+dx) is what specenh_maxpool2_fwd would
 * give; the full-resolution output is never written. Needs bf16/f16, in_dil 1, even
 * OH/OW, no mask/logits/out_f32 (SPECENH_EUNSUPPORTED otherwise). */
int specenh_conv2d(int dtype, const void* in, int N, int IH, int IW, int C, const void* w_gemm,
                   int KH, int KW, int CO, const float* bias, int stride, int pad_t, int pad_l,
                   int in_dil, int OH, int OW, int act, const void* mask, float* logits,
                   void* out, int out_f32, int pool2, unsigned char* argmax, void* stream);
/* Weight gradient of the same convolution: dw[co][k] += sum_m dout[m][co] * A[m][k]
 * (fp32, w_gemm layout, accumulated), dbias[co] += sum_m dout[m][co] (optional). Deterministic: pixel
 * chunks are reduced in a fixed order through `workspace`, which must hold
 * specenh_conv2d_wgrad_workspace_bytes(N, OH, OW, KH, KW, C, CO) bytes. */
size_t specenh_conv2d_wgrad_workspace_bytes(int N, int OH, int OW, int KH, int KW, int C,
                                            int CO);
int specenh_conv2d_wgrad(int dtype, const void* in, int N, int IH, int IW, int C,
                         const void* dout, int KH, int KW, int CO, int stride, int pad_t,
                         int pad_l, int in_dil, int OH, int OW, float* dw, float* dbias,
                         void* workspace, void* stream);
/* specenh_conv2d_wgrad with overwrite != 0: dw and dbias are OVERWRITTEN with the gradient
 * (same values as accumulating into zeroed buffers; Model.fit's layers each own their slice
 * of the gradient buffer, so no zeroing launch precedes them). */
int specenh_conv2d_wgrad_ex(int dtype, const void* in, int N, int IH, int IW, int C,
                            const void* dout, int KH, int KW, int CO, int stride, int pad_t,
                            int pad_l, int in_dil, int OH, int OW, float* dw, float* dbias,
                            int overwrite, void* workspace, void* stream);
/* specenh_conv2d_wgrad of a convolution followed by ReLU + MaxPooling2D((2,2)), given the
 * POOL's output gradient dpool [N][OH/2][OW/2][CO] instead of dout: dout is what
 * specenh_maxpool2_bwd(dpool, argmax, pooled) would write (the gradient routed to the argmax,
 * zero where pooled <= 0; pooled may be NULL: no ReLU mask), formed while the tiles are staged
 * (the model's first Conv2D in Model.fit, manual_scan_3layers.py:187-188: no full-resolution
 * gradient is written; round 6: also the pooled Conv2Ds after it, :190-193). bf16 / f16,
 * C = 1 or C % 16 == 0, stride 1, even OH / OW, CO % 8 == 0, else SPECENH_EUNSUPPORTED. Same
 * workspace as specenh_conv2d_wgrad, but dw and dbias are OVERWRITTEN with the gradient (not
 * accumulated: no zeroing launch before it). */
int specenh_conv2d_wgrad_pooled(int dtype, const void* in, int N, int IH, int IW, int C,
                                const void* dpool, const unsigned char* argmax, const void* pooled,
                                int KH, int KW, int CO, int stride, int pad_t, int pad_l,
                                int in_dil, int OH, int OW, float* dw, float* dbias,
                                void* workspace, void* stream);
/* specenh_conv2d (stride 1, in_dil 1, no pool2 / logits / out_f32) of an input that is the
 * full-resolution gradient of a ReLU + MaxPooling2D((2,2)), given as the POOL's output
 * gradient dpool [N][IH/2][IW/2][C], its argmax and pooled output (pooled may be NULL: no ReLU
 * mask): in = what specenh_maxpool2_bwd(dpool, argmax, pooled) would write, formed while the
 * input patches are staged — the input gradient of a pooled Conv2D in Model.fit
 * (manual_scan_3layers.py:188-193) without the full-resolution gradient tensor or the pool
 * backward launch. Bitwise the pool backward followed by specenh_conv2d. bf16 / f16, even
 * IH / IW, C % 16 == 0 (else SPECENH_EUNSUPPORTED); mask, bias and act as specenh_conv2d. */
int specenh_conv2d_pooled_in(int dtype, const void* dpool, const unsigned char* argmax,
                             const void* pooled, int N, int IH, int IW, int C, const void* w_gemm,
                             int KH, int KW, int CO, const float* bias, int pad_t, int pad_l,
                             int OH, int OW, int act, const void* mask, void* out, void* stream);
/* MaxPooling2D((2,2), padding="same") on even H, W: out [N][H/2][W/2][C] + argmax (0..3). */
int specenh_maxpool2_fwd(int dtype, const void* in, int N, int H, int W, int C, void* out,
                         unsigned char* argmax, void* stream);
/* din [N][H][W][C] = dout routed to the argmax; when pooled (the pool's output, same shape
 * as dout) is given, positions with pooled <= 0 get 0 — the ReLU mask of the pool's input
 * at its argmax. */
int specenh_maxpool2_bwd(int dtype, const void* dout, const unsigned char* argmax,
                         const void* pooled, int N, int H, int W, int C, void* din,
                         void* stream);
/* binary_crossentropy after a sigmoid, from the fp32 logits z (Keras graph mode):
 * *loss_sum += sum_i max(z,0) - z t + log1p(exp(-|z|)) (fp64, zero it first);
 * grad (optional) = (sigmoid(z) - t) / n in grad_dtype. */
int specenh_bce_logits(const float* z, const void* target, int target_dtype, long long n,
                       void* grad, int grad_dtype, double* loss_sum, void* stream);
/* Keras Adam on fp32 master weights, with g = grad_scale * grad (1/world_size after a
 * summing all-reduce): m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2,
 * w -= lr_t m / (sqrt(v) + eps); w_lowp (optional) receives w in lowp_dtype (BF16/F16). */
int specenh_adam_step(float* w, const float* g, float* m, float* v, long long n, float lr_t,
                      float b1, float b2, float eps, float grad_scale, void* w_lowp,
                      int lowp_dtype, void* stream);
/* specenh_adam_step, and in the same pass the input-gradient GEMM weights of nseg (<= 8)
 * layers from the updated weights: segment s is w[seg_off[s] .. + k k ci co) as forward GEMM
 * weights [co][k][k][ci] (seg_kcc[3s .. 3s+2] = k, ci, co); seg_dst[s] ([ci][k][k][co], in
 * lowp_dtype, fp32 when w_lowp is NULL) receives specenh_weight_flip_transpose of the updated
 * copy. One launch instead of an Adam launch plus one flip launch per layer. */
int specenh_adam_step_flip(float* w, const float* g, float* m, float* v, long long n, float lr_t,
                           float b1, float b2, float eps, float grad_scale, void* w_lowp,
                           int lowp_dtype, int nseg, const long long* seg_off, const int* seg_kcc,
                           void* const* seg_dst, void* stream);
/* bd[i][a][b][o] = bt[o][k-1-a][k-1-b][i] (bt: [co][k][k][ci], bd: [ci][k][k][co]):
 * the GEMM weights of a convolution's input gradient from its forward GEMM weights. */
int specenh_weight_flip_transpose(int dtype, const void* bt, int k, int ci, int co, void* bd,
                                  void* stream);
/* Element conversion between f32, bf16 and f16 (round to nearest even). */
int specenh_cast(int src_dtype, const void* src, int dst_dtype, void* dst, long long n,
                 void* stream);

/* The model's last two layers fused for inference (manual_scan_3layers.py:197-199):
 *   Conv2DTranspose(CO, kt, strides=2, activation="relu", padding="same") on x [N][H][W][C]
 *   -> Conv2D(1, ko, activation="sigmoid", padding="same") -> out fp32 [N][2H][2W]
 * with wt_gemm / bt and wo_gemm / bo the two layers' specenh_conv2d weights (GEMM layout,
 * dtype) and fp32 biases (device pointers). The CO-channel map between the layers stays
 * in LDS; it is rounded to dtype after the ReLU exactly as the two-launch path stores it.
 * dtype BF16 / F16; C = 32 with CO = 16, kt = ko = 5 (the reference model,
 * manual_scan_3layers.py:197-199), or, on W = 64 inputs, CO = 32, kt = ko in {3, 5, 7} (the
 * 32/32 models of hyperparam_scan.py:160-162 at their 256 x 128 inputs) or CO = 64,
 * kt = ko in {3, 5} (manual_scan.py:198-199); otherwise
 * SPECENH_EUNSUPPORTED (use the two specenh_conv2d launches). */
int specenh_convt_conv_out(int dtype, const void* x, int N, int H, int W, int C,
                           const void* wt_gemm, const float* bt, int CO, int kt,
                           const void* wo_gemm, const float* bo, int ko, float* out,
                           void* stream);

/* Training form of specenh_convt_conv_out (Model.fit's forward through the same two layers,
 * manual_scan_3layers.py:197-199, :213): the row-sweep launch also stores the ReLU'd CO-channel
 * map (dtype [N][2H][2W][CO]: the backward's ReLU mask and weight-gradient input; the same
 * products as the unfused Conv2DTranspose summed in a different fp32 order, so a few elements
 * can differ from its store by one rounding step of dtype, and training is not bitwise the
 * unfused path's: SPECENH_NO_TAIL_TRAIN=1 selects the two launches when bitwise parity with
 * them is needed), the fp32 logits [N][2H][2W] (the BCE input)
 * and the sigmoid output in dtype [N][2H][2W]. W = 64 only (the reference model at 128 x 128),
 * else SPECENH_EUNSUPPORTED (use the two specenh_conv2d launches). */
int specenh_convt_conv_out_train(int dtype, const void* x, int N, int H, int W, int C,
                                 const void* wt_gemm, const float* bt, int CO, int kt,
                                 const void* wo_gemm, const float* bo, int ko, void* map,
                                 float* logits, void* out, void* stream);

/* The decoder's last THREE layers in one launch (VAE/manual_scan_3layers.py:196-199, the
 * inference path of predict :239):
 *   x [N][H][W][C] -> Conv2DTranspose(CO1, k, strides=2, relu, "same")
 *                  -> Conv2DTranspose(CO2, k, strides=2, relu, "same")
 *                  -> Conv2D(1, k, sigmoid, "same") -> out fp32 [N][4H][4W]
 * w1_gemm / b1, wt_gemm / bt, wo_gemm / bo: the three layers' specenh_conv2d weights (GEMM
 * layout, dtype) and fp32 biases. Both intermediate maps stay in LDS, each rounded to dtype
 * after its ReLU exactly as the unfused path stores it. dtype BF16 / F16; W = 32, C = 64,
 * CO1 = 32, CO2 = 16, k = 5 (the reference model on 128 x 128 inputs), otherwise
 * SPECENH_EUNSUPPORTED. */
int specenh_decoder3(int dtype, const void* x, int N, int H, int W, int C,
                     const void* w1_gemm, const float* b1, int CO1, const void* wt_gemm,
                     const float* bt, int CO2, const void* wo_gemm, const float* bo, int k,
                     float* out, void* stream);
/* specenh_decoder3 with the output precision selectable: out_dtype F32 (float [N][4H][4W]) or
 * F16 (_Float16, the sigmoid rounded once: BASELINE config 5's 32,768-byte fp16
 * reconstruction per 128 x 128 shot). */
int specenh_decoder3_ex(int dtype, const void* x, int N, int H, int W, int C,
                        const void* w1_gemm, const float* b1, int CO1, const void* wt_gemm,
                        const float* bt, int CO2, const void* wo_gemm, const float* bo, int k,
                        void* out, int out_dtype, void* stream);

/* The encoder's first TWO layers in one launch (VAE/manual_scan_3layers.py:187-191, the
 * inference path of predict :239):
 *   x [N][H][W][1] -> Conv2D(CO1, k, relu, "same") -> MaxPooling2D(2)
 *                  -> Conv2D(CO2, k, relu, "same") -> MaxPooling2D(2) -> out [N][H/4][W/4][CO2]
 * w1_gemm / b1, w2_gemm / b2: the two layers' specenh_conv2d weights (GEMM layout, dtype) and
 * fp32 biases. The pooled CO1-channel map stays in LDS, rounded to dtype after its ReLU
 * exactly as the unfused path stores it. dtype BF16 / F16; W = 128, CO1 = 16, CO2 = 32,
 * k = 5, H a multiple of 4, x 16-byte aligned (the reference model on 128 x 128 inputs),
 * otherwise SPECENH_EUNSUPPORTED / SPECENH_EINVAL. */
int specenh_encoder2(int dtype, const void* x, int N, int H, int W, const void* w1_gemm,
                     const float* b1, int CO1, const void* w2_gemm, const float* b2, int CO2,
                     int k, void* out, void* stream);

/* ---------------------------------------------------------------- label filters
 * The image-filter helpers of spec_denoising/pipeline_data.py:38-61 (the training-label
 * chain) on a batch of spectrograms, each a rows x cols row-major block at
 * S + b*stride (dtype SPECENH_DTYPE_F32 or _F64; out may alias S). Statistics are per
 * spectrogram, accumulated in fp64:
 *   SPECENH_FILTER_NORM     (x - mean) / std                 norm,     :38-41 (np.std, ddof 0)
 *   SPECENH_FILTER_RESCALE  (x - min) / (max - min)          rescale,  :43-44
 *   SPECENH_FILTER_MEANSUB  rescale(|x - mean of its row|)   meansub,  :58-61
 * workspace >= specenh_filter_workspace_bytes(batch, rows).
 * specenh_quantfilt: x < q(column) ? 0 : x with q the numpy 'linear' thr-quantile of each
 * column (np.quantile(src, thr, axis=0), quantfilt :46-49); rows <= 1264. */
#define SPECENH_FILTER_NORM 0
#define SPECENH_FILTER_RESCALE 1
#define SPECENH_FILTER_MEANSUB 2
size_t specenh_filter_workspace_bytes(long long batch, int rows);
int specenh_filter(int op, int dtype, const void* S, long long batch, int rows, int cols,
                   long long stride, void* out, void* workspace, void* stream);
int specenh_quantfilt(int dtype, const void* S, long long batch, int rows, int cols,
                      long long stride, double thr, void* out, void* stream);

/* gaussblr / morph (pipeline_data.py:52-55, :64-72): each spectrogram is
 * quantised to uint8 as (rescale(x)*255).astype('uint8'), filtered with OpenCV's 8-bit
 * algorithms restated (cv2 is absent: parity with cv2 unpinned, restatement in
 * oracle/filters.py), and rescaled to [0, 1] as numpy does on a uint8 array:
 *   specenh_gaussblr: cv2.GaussianBlur(u8, (kw, kh), sigma) — kw taps along cols, kh along
 *                     rows, odd sizes <= 127, sigma <= 0 derives it from the size;
 *                     integer Q8 taps, BORDER_REFLECT_101 (reference call: (31, 3), 0).
 *   specenh_morph:    MORPH_CLOSE with a 4x4 rect, then MORPH_OPEN with a 3x1 (w x h) rect.
 * workspace >= specenh_u8filter_workspace_bytes(batch, rows, cols). */
size_t specenh_u8filter_workspace_bytes(long long batch, int rows, int cols);
int specenh_gaussblr(int dtype, const void* S, long long batch, int rows, int cols,
                     long long stride, int kw, int kh, double sigma, void* out, void* workspace,
                     void* stream);
int specenh_morph(int dtype, const void* S, long long batch, int rows, int cols, long long stride,
                  void* out, void* workspace, void* stream);

/* ---------------------------------------------------------------- strip glue
 * patch / unpatch / reshape of VAE/manual_scan_3layers.py:28-54:
 *   pack:   out[(b*n_strips + x)][r][c] = S[b][r][x*width + c], r < rows, c < width
 *           (S: fp32 [batch][F][T] at S + b*s_stride; out: dst_dtype, i.e. the AE's NHWC
 *           input with C = 1). Reference values: rows 256, width 128, n_strips 30.
 *   unpack: out[b][r][x*width + c] = strips[(b*n_strips + x)][r][c] (fp32 out).
 * width must be a multiple of 4. */
int specenh_strips_pack(int dst_dtype, const float* S, long long batch, int F, int T,
                        long long s_stride, int rows, int width, int n_strips, void* out,
                        void* stream);
int specenh_strips_unpack(int src_dtype, const void* strips, long long batch, int rows, int width,
                          int n_strips, float* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SPECENH_H */
