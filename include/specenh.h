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

/* Output-mode flags for specenh_stft_psd. */
#define SPECENH_STFT_LOG 1          /* natural log(P + eps)                  pipeline_data.py:33 */
#define SPECENH_STFT_NORMALIZE 2    /* per-spectrogram min-max (implies LOG) pipeline_data.py:34 */
#define SPECENH_STFT_DROP_NYQUIST 4 /* drop the last frequency row         pipeline_data.py:35 */

/* detrend / scaling codes (the 'detrend' and 'scaling' keys of spec_params,
 * pipeline_data.py:77-84). */
#define SPECENH_DETREND_NONE 0
#define SPECENH_DETREND_CONSTANT 1
#define SPECENH_DETREND_LINEAR 2
#define SPECENH_SCALING_DENSITY 0
#define SPECENH_SCALING_SPECTRUM 1

const char* specenh_last_error(void);
const char* specenh_version(void);

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

/* ---------------------------------------------------------------- SVD denoiser
 * Batched replacement for denoiseSignal(matrix, start, stop, use_optimal=False)
 * (spec_denoising/denoising_by_svd.ipynb:188-229):
 *   u, s, vh = np.linalg.svd(A, full_matrices=False)
 *   out = u[:, start:stop] @ diag(s[start:stop]) @ vh[start:stop, :]
 * with the notebook's clamping (start < 0 -> 0, stop > r -> r, r = min(m, n)) and
 * start >= stop -> zeros. A: device fp32, matrix b at A + b*a_stride, row-major m x n.
 * out: device fp32 [batch][m][n]. The top-K singular subspace it needs (K = stop, or
 * start when stop == r) must satisfy K <= 40 (SPECENH_EUNSUPPORTED otherwise).
 * workspace: >= specenh_svd_workspace_bytes(batch, m, n, K) bytes. */
size_t specenh_svd_workspace_bytes(long long batch, int m, int n, int kmax);
int specenh_svd_denoise(const float* A, long long batch, int m, int n, long long a_stride,
                        int start, int stop, float* out, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SPECENH_H */
