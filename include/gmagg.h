/*
 * gmagg.h — C ABI of the MI355X geometric-median aggregation library
 * (libgmagg.so, built from byzantine_aircomp_amd/csrc/ for gfx950).
 *
 * This is the drop-in boundary for the reference's aggregation call
 *     weight_vector = aggregate(weight_f, options)          MNIST_Air_weight.py:353
 * with aggregate resolved by eval(args.agg) (MNIST_Air_weight.py:580).  Each entry
 * point below names the reference function it replaces.  Plain pointers and
 * sizes only: no torch types cross this boundary.
 *
 * Conventions
 *   - Every call returns 0 (GM_OK) or a negative GM_ERR_* code; the message of
 *     the last failure on the calling thread is gm_last_error().  Nothing aborts
 *     or throws across the ABI.
 *   - Device pointers are HIP device pointers on the context's device; the
 *     caller owns X / guess / out, the library owns its workspace.
 *   - Work is stream-ordered on `stream` (a hipStream_t passed as void*; NULL =
 *     the default stream).  gm_weiszfeld_f32 blocks only to learn whether the
 *     iteration has converged; the OMA entry points never block.
 *   - A context is used by one host thread at a time.  Calls on one context may
 *     use different streams: each call makes its stream wait for the previous
 *     call's queued work on the context's workspace (an event), so they never
 *     race; for concurrent aggregations use one context per stream.
 *
 * Layout: X is row-major [K][ldx] fp32, row k = client k's flattened update
 * (model.parameters() order, MNIST_Air_weight.py:206-209), ldx >= d — the
 * reference's own torch.stack layout.  gm_weiszfeld_f32 also takes the panel
 * layout (gm_opts.layout = GM_LAYOUT_PANELS): X as [ceil(d/W)][K][W] with
 * W = gm_panel_width(K) and ldx = elements between panels (>= K*W); element
 * (k, j) at X[(j/W)*ldx + k*W + j%W].  Each streaming-pass chunk is then one
 * contiguous block of HBM.
 */
#ifndef GMAGG_H
#define GMAGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GMAGG_ABI_VERSION 4

enum gm_status {
    GM_OK = 0,
    GM_ERR_INVALID = -1,      /* bad argument (null pointer, negative size, ...) */
    GM_ERR_HIP = -2,          /* a HIP runtime call failed */
    GM_ERR_UNSUPPORTED = -3,  /* shape / mode this build does not handle */
    GM_ERR_CALLBACK = -4,     /* a user callback (noise, all-reduce) returned non-zero */
    GM_ERR_COMM = -5          /* RCCL failure */
};

enum gm_mode {
    GM_MODE_IDEAL = 0,        /* gm2: MNIST_Air_weight.py:162-184 */
    GM_MODE_AIRCOMP = 1       /* gm + OMA2 per iteration: MNIST_Air_weight.py:131-160, 396-414 */
};

enum gm_noise_source {
    GM_NOISE_PHILOX = 0,      /* on-device Philox4x32-10, keyed (seed, iteration, global index) */
    GM_NOISE_HOST = 1         /* caller supplies the reference's draws through noise_cb */
};

enum gm_layout {
    GM_LAYOUT_ROWS = 0,       /* [K][ldx] row-major (the reference's torch.stack of rows) */
    GM_LAYOUT_PANELS = 1      /* [ceil(d/W)][K][W], W = gm_panel_width(K), ldx = panel stride;
                                 streaming, (gm2, K <= 256, W % 64 == 0) the guarded Gram, or
                                 (K <= 52 gm2 / K <= 50 gm, unsharded) the resident kernel */
};

enum gm_algo {
    GM_ALGO_AUTO = 0,
    GM_ALGO_STREAM = 1,       /* fused one-read-per-iteration streaming Weiszfeld */
    GM_ALGO_TWOPASS = 2,      /* two reads per iteration; any K */
    GM_ALGO_GRAM = 3,         /* K x K Gram on MFMA, iterations in K-space (IDEAL only, K <= 256):
                                 scaled f16 hi/lo split, 3 v_mfma_f32_32x32x16_f16 products per
                                 off-diagonal tile (2 on the diagonal); an f16 range overflow
                                 reruns the bf16 h+m split (4 products, rows) or the streaming
                                 path (panels); the result is kept only if the a-posteriori
                                 guard passes (gm_result.guard / gram_kind) */
    GM_ALGO_RESIDENT = 4,     /* small problems: X held in VGPRs, all iterations in one launch */
    GM_ALGO_GRAM_F32 = 5      /* the Gram on the exact f32-input MFMA (4x the issue cycles) */
};

/* Host-noise callback for GM_NOISE_HOST: fill the draws of Weiszfeld iteration
 * `iter` (0-based), exactly as OMA2 draws them (MNIST_Air_weight.py:401-402, 411):
 * h_re[K], h_im[K] ~ N(0, 1/2) and, when the options ask for noise,
 * noise[d_total + 1] ~ N(0, noise_var / 2) (the last element is the
 * denominator's).  Buffers are host memory owned by the library.  Return 0. */
typedef int (*gm_noise_cb)(void* user, int64_t iter, float* h_re, float* h_im, float* noise);

/* Optional d-sharding hook: sum `count` doubles in place across all shards,
 * stream-ordered on `stream`.  Return 0.  (gm_ctx_init_rccl installs a native
 * RCCL all-reduce instead.) */
typedef int (*gm_allreduce_cb)(void* user, double* dev_buf, int64_t count, void* stream);

typedef struct gm_opts {
    int64_t maxiter;          /* options['maxiter'], reference default 200 (M:136, M:167) */
    double tol;               /* options['tol'], default 1e-5; compared as fp32 like the reference */
    double eps;               /* distance floor, 1e-4 in the reference (M:151, M:178) */
    int32_t mode;             /* gm_mode */
    int32_t has_noise;        /* AIRCOMP: options['noise_var'] is not None */
    double noise_var;         /* AIRCOMP: channel-noise variance (OMA2 std = sqrt(var/2), M:410) */
    double P_max;             /* AIRCOMP: options['P_max'], default 1 (M:136) */
    uint64_t seed;            /* GM_NOISE_PHILOX key */
    int32_t noise_source;     /* gm_noise_source */
    int32_t algo;             /* gm_algo */
    gm_noise_cb noise_cb;     /* GM_NOISE_HOST */
    void* noise_user;
    int32_t check_every;      /* host convergence poll interval in iterations; 0 = auto */
    int32_t layout;           /* gm_layout of X (gm_weiszfeld_f32 and gm_weiszfeld_batched_f32) */
    /* pre_oma = 1 (gm2 only): first apply OMA(X, pre_oma_var) IN PLACE, as the reference
     * does before every non-gm aggregator when --var is set (MNIST_Air_weight.py:351-352),
     * with the draws of gm_oma_philox_f32 (batched: problem p keyed pre_oma_seed + p *
     * 0x9E3779B97F4A7C15).  The streaming path fuses it into its first pass. */
    int32_t pre_oma;
    double pre_oma_var;
    uint64_t pre_oma_seed;
} gm_opts;

enum gm_guard {
    GM_GUARD_NONE = 0,        /* no Gram result was involved */
    GM_GUARD_ACCEPTED = 1,    /* Gram-space result, a-posteriori accuracy guard passed */
    GM_GUARD_REJECTED = 2,    /* a Gram result was refused; the streaming path produced out */
    GM_GUARD_ACCEPTED_FLOOR = 3 /* accepted, with tol inside the reference's fp32 movement
                                 floor band (tol/3 < 2^-23 ||g|| <= tol): any fp32 Weiszfeld's
                                 count is decided by rounding there; iters is the exact count */
};

enum gm_exchange {
    GM_EXCHANGE_NONE = 0,      /* launch-per-pass paths: partials reduced between launches */
    GM_EXCHANGE_AGENT = 1,     /* resident grid over several XCDs: agent-scope granule stores */
    GM_EXCHANGE_XCD_LOCAL = 2, /* resident grid on ONE XCD (confirmed from XCC_ID at the
                                  check-in): granules kept in that XCD's L2 */
    GM_EXCHANGE_XCD_HIER = 3,  /* resident grid over several XCDs, gathered per XCD: each
                                  block's granules kept in its XCD's L2 for the XCD's leader,
                                  the 8 per-XCD sums exchanged agent-scope */
    GM_EXCHANGE_XCD_SPLIT = 4  /* resident grid over several XCDs, one hop: each granule stored
                                  agent-scope and L2-kept, a reader polling its own XCD's
                                  blocks from the L2-kept copies */
};

typedef struct gm_result {
    int64_t iters;            /* Weiszfeld loop bodies executed (M:145 / M:173) */
    double last_movement;     /* ||guess_t - guess_{t+1}|| of the last body (M:156 / M:180) */
    int32_t converged;        /* 1 if the loop exited through the tol test */
    int32_t algo_used;        /* gm_algo actually run */
    int32_t guard;            /* gm_guard: what the Gram accuracy guard decided */
    int32_t gram_kind;        /* Gram runs: 1 scaled f16 split (3 MFMA products), 2 bf16 split
                                 (4 products, after an f16 range overflow), 3 f32-input; else 0 */
    int32_t exchange;         /* register-resident runs: how the blocks exchanged their
                                 per-iteration partials (gm_exchange); else GM_EXCHANGE_NONE */
} gm_result;

typedef struct gm_ctx gm_ctx;

/* Context: device binding, workspace, optional shard description. */
int gm_ctx_create(int device, gm_ctx** out);
int gm_ctx_destroy(gm_ctx* ctx);

/* d-sharding: this shard holds global columns [d_offset, d_offset + d_local) of
 * a d_total-long update; per-iteration partial sums go through the all-reduce.
 * Every rank must pass the same K, d_total and options; the library takes every
 * decision that changes the sequence of collectives (Gram or streaming, the poll
 * interval) from those global values, so a shorter or ragged last shard issues
 * exactly the all-reduces the others do.  For AUTO's Gram choice (gm2, K <= 256,
 * d_total >= 2^18, d_total % 4 == 0) each shard must also be 16-byte aligned with
 * d_local and ldx multiples of 4 — always true for contiguous shards cut at
 * 256-column boundaries (byzantine_aircomp_amd.sharded.shard_range). */
int gm_ctx_set_shard(gm_ctx* ctx, int64_t d_total, int64_t d_offset);
int gm_ctx_set_allreduce(gm_ctx* ctx, gm_allreduce_cb fn, void* user);
/* Native RCCL all-reduce over xGMI: `unique_id` is the 128-byte ncclUniqueId
 * made by rank 0 (gm_rccl_get_unique_id) and shared by the caller. */
int gm_rccl_get_unique_id(void* unique_id_128);
int gm_ctx_init_rccl(gm_ctx* ctx, const void* unique_id_128, int nranks, int rank);

/* gm2 / gm: Weiszfeld geometric median of the K rows of X.
 * Replaces gm2(wList, options) (MNIST_Air_weight.py:162-184) with
 * opts->mode = GM_MODE_IDEAL, and gm(wList, options) (MNIST_Air_weight.py:131-160,
 * calling OMA2 M:396-414 each iteration) with GM_MODE_AIRCOMP.
 * guess0 = options['guess'] (d floats); out receives the returned iterate
 * (d floats).  maxiter == 0 copies guess0 to out. */
int gm_weiszfeld_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t ldx,
                     const float* guess0, float* out, const gm_opts* opts,
                     gm_result* result, void* stream);

/* Panel width W of the GM_LAYOUT_PANELS layout for K clients (the streaming
 * tile's chunk width: 32 columns at 512 < K <= 1024); 0 if K is unsupported. */
int64_t gm_panel_width(int64_t K);

/* Batched independent problems (BASELINE config C5, the draw.ipynb-style sweep
 * over many small aggregations): problem p aggregates the K rows at X + p*ldp
 * (row stride ldx) from guess0 + p*ldg into out + p*ldo.  One launch per pass
 * covers all P problems; each stops at its own tol test (gm2) or runs maxiter
 * (gm).  Options are shared; GM_MODE_AIRCOMP uses Philox only, problem p keyed
 * with seed + p * 0x9E3779B97F4A7C15.  results: P entries or NULL.  Not
 * combinable with d-sharding.  opts->layout = GM_LAYOUT_PANELS: problem p at X + p*ldp
 * is in the panel layout [ceil(d/W)][K][W] (W = gm_panel_width(K)) with panel stride
 * ldx >= K*W, ldp >= ceil(d/W)*ldx; the same results as the row-major call. */
int gm_weiszfeld_batched_f32(gm_ctx* ctx, const float* X, int64_t P, int64_t K, int64_t d,
                             int64_t ldx, int64_t ldp, const float* guess0, int64_t ldg,
                             float* out, int64_t ldo, const gm_opts* opts, gm_result* results,
                             void* stream);

/* The reference's other aggregators (MNIST_Air_weight.py:186-204), out[d]:
 *   gm_mean_f32          mean(wList, options)          M:186-187
 *   gm_median_f32        median(wList, options)        M:194-195 (lower median), K <= 2048
 *   gm_trimmed_mean_f32  trimmed_mean(wList, options)  M:189-192, trim = int(0.1 K) per end, K <= 2048
 *   gm_krum_f32          Krum(wList, options)          M:197-204, K <= 4096; *index = chosen row
 * Larger K returns GM_ERR_UNSUPPORTED. */
int gm_mean_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                void* stream);
int gm_median_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                  void* stream);
int gm_trimmed_mean_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t ldx,
                        int64_t trim, float* out, void* stream);
int gm_krum_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t ldx,
                int64_t honest_size, float* out, int64_t* index, void* stream);
/* The same four on client updates in the panel layout (GM_LAYOUT_PANELS: X as
 * [ceil(d/W)][K][W], W = gm_panel_width(K), panel_stride >= K*W): identical results. */
int gm_mean_panels_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t panel_stride,
                       float* out, void* stream);
int gm_median_panels_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t panel_stride,
                         float* out, void* stream);
int gm_trimmed_mean_panels_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d,
                               int64_t panel_stride, int64_t trim, float* out, void* stream);
int gm_krum_panels_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t panel_stride,
                       int64_t honest_size, float* out, int64_t* index, void* stream);

/* Krum's algorithm (round 5).  K <= 256 on large inputs (AUTO: K >= 64 and K^2 d >= 2^29;
 * env GMAGG_KRUM=0 exact only, 1 Gram wherever eligible): the scaled-f16 Gram MFMA kernel
 * gives every pairwise distance within a stated bound, rows whose score bounds reach the
 * smallest upper bound are recomputed with the exact path's arithmetic, and the index equals
 * the exact path's.  gm_krum_last_info: info[3] = {algorithm, candidates recomputed,
 * reason} of this context's last Krum call. */
enum gm_krum_algo { GM_KRUM_EXACT = 0, GM_KRUM_GRAM = 1 };
enum gm_krum_reason {
  GM_KRUM_REASON_OK = 0,             /* the Gram path ran */
  GM_KRUM_REASON_NOT_CHOSEN = 1,     /* exact by choice (GMAGG_KRUM, AUTO's size rule) */
  GM_KRUM_REASON_NOT_ELIGIBLE = 2,   /* K > 256, misaligned rows, d or ldx % 4, panel width */
  GM_KRUM_REASON_GRAM_NONFINITE = 3, /* the f16 range was exceeded or the input is not finite */
  GM_KRUM_REASON_CANDIDATES = 4      /* more than 128 candidates, or a bound not finite */
};
int gm_krum_last_info(gm_ctx* ctx, int64_t* info);

/* getVarience(w_local, honestSize) (MNIST_Air_weight.py:127-129): the mean over the
 * first `honest` rows of ||x_k - mean||^2, written as ONE fp32 value to the device
 * pointer `out`; one streaming pass over the honest rows (fp64 sums). */
int gm_honest_variance_f32(gm_ctx* ctx, const float* X, int64_t honest, int64_t d, int64_t ldx,
                           float* out, void* stream);
/* The same on a client matrix of K rows in the panel layout (GM_LAYOUT_PANELS). */
int gm_honest_variance_panels_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t honest,
                                  int64_t d, int64_t panel_stride, float* out, void* stream);

/* OMA(message, noise_var): in-place per-client equalised AWGN
 * (MNIST_Air_weight.py:385-394), draws from on-device Philox keyed by `seed`. */
int gm_oma_philox_f32(gm_ctx* ctx, float* X, int64_t K, int64_t d, int64_t ldx,
                      double noise_var, uint64_t seed, void* stream);

/* OMA on P independent problems X[p] = X + p*pstride ([K][ldx] each; BASELINE C5,
 * the reference's `--agg gm2 --var v` pre-noise, MNIST_Air_weight.py:351-352):
 * problem p's draws are gm_oma_philox_f32's with seed + p * 0x9E3779B97F4A7C15. */
int gm_oma_philox_batched_f32(gm_ctx* ctx, float* X, int64_t P, int64_t K, int64_t d, int64_t ldx,
                              int64_t pstride, double noise_var, uint64_t seed, void* stream);

/* Batched OMA on P problems in the panel layout: problem p at X + p*pstride is
 * [ceil(d/W)][K][W] with panel_stride >= K*W; the same draws as
 * gm_oma_philox_batched_f32 on the row-major problems. */
int gm_oma_philox_batched_panels_f32(gm_ctx* ctx, float* X, int64_t P, int64_t K, int64_t d,
                                     int64_t panel_stride, int64_t pstride, double noise_var,
                                     uint64_t seed, void* stream);

/* The same OMA on client updates in the panel layout (GM_LAYOUT_PANELS: X as
 * [ceil(d/W)][K][W], W = gm_panel_width(K), panel_stride >= K*W): identical draws
 * and results to gm_oma_philox_f32 on the row-major matrix; padding untouched. */
int gm_oma_philox_panels_f32(gm_ctx* ctx, float* X, int64_t K, int64_t d, int64_t panel_stride,
                             double noise_var, uint64_t seed, void* stream);

/* Caller-side packing (row f2): copy the row-major client matrix X[K][ldx] (the
 * reference's flatten_list stack, MNIST_Air_weight.py:206-209) into the panel layout
 * P = [ceil(d/W)][K][W] with panel_stride >= K*W elements between panels
 * (GM_LAYOUT_PANELS).  Padding columns >= d are not written. */
int gm_rows_to_panels_f32(gm_ctx* ctx, const float* X, int64_t K, int64_t d, int64_t ldx,
                          float* P, int64_t W, int64_t panel_stride, void* stream);

/* The K clients' local SGD steps of one federated step (the loop body M:291-343:
 * forward, CrossEntropyLoss (mean), backward, p -= gamma * (grad + weight_decay * p),
 * the client's parameters copied out as its row), as one stream-ordered kernel, for the
 * reference's linear model MLP(F, C) (M:53-61; F <= 832, C <= 64, batch B <= 64).
 * The clients run in sequence on ONE model, as the reference's aliasing state_dict
 * "snapshot" makes them (M:290, M:343): client k starts from client k-1's update, and
 * W / b end as the last client's parameters (the aggregator's guess, M:349).
 *   data     training samples [n][ldd] fp32 (device), labels [n] int64 (device)
 *   idx      [K][B] int32 dataset rows of each client's batch (device): the reference's
 *            RandomSampler draws (M:260-270), offset by the client's shard start
 *   honest   clients k >= honest are Byzantine: attack 1 = classflip (target C-1-y,
 *            M:320), 2 = dataflip (input 1-x, M:326), 0 = none (also weightflip,
 *            which rewrites the matrix afterwards, M:380-383)
 *   W, b     the model's weight [C][F] and bias [C] (device), updated in place
 *   X        the client matrix: row k = [W (C*F, row-major), b (C)], layout
 *            GM_LAYOUT_ROWS (ldx = row stride >= C*F + C) or GM_LAYOUT_PANELS
 *            (ldx = panel stride >= K*W, W = gm_panel_width(K)). */
int gm_client_chain_f32(gm_ctx* ctx, const float* data, int64_t ldd, const int64_t* labels,
                        int64_t F, int64_t C, const int32_t* idx, int64_t K, int64_t B,
                        int64_t honest, int32_t attack, float gamma, float weight_decay,
                        float* W, float* b, float* X, int64_t ldx, int32_t layout, void* stream);

/* OMA with the reference's own draws (device arrays): h_re[K], h_im[K],
 * n_re[K*d], n_im[K*d] (row-major, already scaled by sqrt(noise_var)).
 * Bit-exact with the reference's fp32 op order. */
int gm_oma_apply_f32(gm_ctx* ctx, float* X, int64_t K, int64_t d, int64_t ldx,
                     const float* h_re, const float* h_im, const float* n_re,
                     const float* n_im, void* stream);

/* Fill X[K][ldx] (first d columns) with seeded synthetic client updates on the
 * device: rows k < K - B ~ N(mu_h, sd_h^2), the last B rows ~ N(mu_b, sd_b^2)
 * (BASELINE.md §3 recipe), Philox-keyed so every shard generates its own
 * columns of the same global matrix (global column = d_offset + j). */
int gm_fill_clients_f32(gm_ctx* ctx, float* X, int64_t K, int64_t d, int64_t ldx, int64_t B,
                        float mu_h, float sd_h, float mu_b, float sd_b, uint64_t seed,
                        void* stream);
/* Fill v[n] ~ N(mu, sd^2) (global index = d_offset + i). */
int gm_fill_normal_f32(gm_ctx* ctx, float* v, int64_t n, float mu, float sd, uint64_t seed,
                       void* stream);

/* Timing hook for the dominant kernel: accumulated device time (ms, HIP
 * events on the launch stream) and launch count of the fused Weiszfeld pass
 * since the last reset. */
int gm_ctx_pass_timing(gm_ctx* ctx, int enable, double* total_ms, int64_t* launches);

const char* gm_last_error(void);
int gm_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GMAGG_H */
