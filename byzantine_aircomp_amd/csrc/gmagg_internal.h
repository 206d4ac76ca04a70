// Internal interface between the C-ABI layer (api.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gmk {

constexpr int kTPB = 1024;           // threads per block of the streaming pass
constexpr int kWaves = kTPB / 64;

// Device-resident state of one Weiszfeld call (written by kspace_step, read by
// every kernel's early-exit test and by the host poll).
struct alignas(64) KState {
  int32_t done;          // 1 once the tol test fired (later launches are no-ops)
  int32_t converged;
  int64_t iters;         // loop bodies executed
  double last_movement;  // fp32 movement of the last body, widened
  float a_noise;         // scale of the per-column noise in the next pass (AIRCOMP)
  float s;               // scaler sqrt(mean(g^2)) of the current iterate (AIRCOMP)
  // Gram variant, written by gram_solve for the AUTO accuracy guard (api.hip):
  double guard_q;        // ||X'^T b||: one-step error of the K-space map (gram_verify)
  double guard_r;        // last / previous K-space movement (contraction estimate)
  int32_t gram_bad;      // the reduced Gram has a non-finite entry (f16 overflow or input)
  int32_t pad0;
  double pad1;
};

// Streaming pass configuration: V floats per lane per row, NW waves per
// block, LPR lanes per row segment (chunk width J = LPR*V columns), R rows
// per thread (the block covers NW*(64/LPR)*R rows).
struct PassCfg {
  int V, NW, LPR, R;
  int OCC = 1;   // blocks per CU the kernel's registers are capped for
};

struct PassArgs {
  const float* X;
  int64_t K, d, ldx;
  const float* g_old;     // iterate t (INIT: the initial guess)
  float* g_new;           // iterate t+1 (STEP)
  const float* coef;      // K normalised weights / AirComp coefficients (STEP)
  const KState* st;
  double* slab;           // [gridDim.x][slab_stride] per-block partial sums
  int64_t slab_stride;
  // additive column noise of the AirComp variant (STEP)
  int noise;              // 0 none, 1 Philox, 2 host-supplied column draws
  const float* hnoise;    // noise == 2: local column draws (d floats)
  uint64_t seed;
  int64_t iter;           // Weiszfeld iteration index the pass computes
  int64_t col_off;        // global index of local column 0 (d-sharding)
  // Batched independent problems (BASELINE C5): blockIdx.y = problem p; X,
  // g_old, g_new advance by these element strides, coef by K, st by 1, slab by
  // gridDim.x * slab_stride, the Philox seed by p * kSeedStride.  0 / unused for P = 1.
  int64_t x_ps, gold_ps, gnew_ps;
  // > 0: X is in the panel layout [ceil(d/J)][K][J] with this many elements
  // between panels (J = the tile's chunk width); 0: row-major [K][ldx].
  int64_t panel_stride;
  // MODE 4 (INIT + OMA): the reference's OMA pre-noise (M:351-352, M:385-394) applied to
  // the tile in registers and written back before the INIT distances; Philox keyed by
  // oma_seed (+ p * kSeedStride for batched problem p), draws as gm_oma_philox_f32's
  float oma_sd;
  uint64_t oma_seed;
  // rows_pass only (the row-major gm2 STEP at two blocks per CU): P = the CU count when the
  // grid is two blocks per CU, else 0.  The hardware places block b and block b + P on one
  // CU, so they take adjacent chunks (first_chunk): the CU's two blocks read adjacent 128-B
  // segments of each row at about the same time (round 6: C3 rows STEP 6,844 -> 6,788 us,
  // with identical UTCL1 misses: DRAM / L2 locality; pairing b with b + 8 or b + 16 gains
  // nothing, and on panels the pairing measured 1.6 % slower:
  // profiles/r6s2_rows_chunk_pair_ab.jsonl, r6s2_utcl1_rows_chunk_pair.json)
  int chunk_pair;
};

// The first chunk of block b in a grid-stride walk (chunks b', b' + grid, ...): b itself,
// or with the pairing above 2 (b mod P) + (b / P) for b < 2P (a permutation of [0, grid)
// when 2P divides the grid)
__host__ __device__ inline int64_t first_chunk(int P, int64_t b, int64_t grid) {
  if (P <= 0 || grid % (2 * P) != 0) return b;
  return 2 * ((b / (2 * P)) * P + b % P) + (b / P) % 2;
}

constexpr uint64_t kSeedStride = 0x9E3779B97F4A7C15ull;
// The reference's fp32 movement floor in ulps of ||g|| (M:180: an fp32 norm of a difference
// of fp32 iterates): the Gram guard accepts an exact-arithmetic count only where
// kFloorUlps * 2^-24 * ||g|| <= tol.  The SAME constant as oracle/aggregators.py FLOOR_ULPS
// (the count window the tests check counts against; measured: profiles/r5s1_movement_floor.txt)
constexpr double kFloorUlps = 2.0;

struct KspaceArgs {
  int64_t K, d_total, t;  // t = pass just completed, -1 after the initial pass
  int mode;               // gm_mode
  int has_noise, noise_src;
  float tol, eps;
  double P_max, noise_sd; // noise_sd = sqrt(noise_var / 2) (OMA2, M:410)
  uint64_t seed;
  int do_check, do_coef;
  const double* sums;     // reduced partials (all shards)
  double* r;              // ||x_k||^2, saved at init (AIRCOMP)
  const float* h_re;      // host-noise draws of iteration t+1 (device copies)
  const float* h_im;
  const float* n_last;    // the denominator's noise element
  float* coef;
  KState* st;
  // Batched: blockIdx.x = problem; sums advance by sums_ps, r / coef by K, st by 1.
  int64_t sums_ps;
  int* n_done;            // problems whose tol test has fired (nullable)
  KState* mirror;         // host-mapped copy of *st written at the end (nullable, one problem)
};

// Streaming pass (stream_pass.hip).  mode: 0 step, 1 init, 2 init + ||x_k||^2, 3 Gram
// closing sum, 4 init after OMA pre-noise written back to X (V = 4 tiles).
hipError_t launch_pass(const PassCfg& cfg, int mode, int grid, const PassArgs& a, hipStream_t s,
                       int problems = 1);
int pass_blocks_per_cu(const PassCfg& cfg, int mode);
// The row-major gm2 STEP / INIT at 512 < K <= 1024 on 32 waves per CU (rows_pass.hip).
bool rows_pass_eligible(const PassArgs& a, int mode);
hipError_t launch_rows_pass(int mode, int grid, const PassArgs& a, hipStream_t s);
bool pass_cfg_supported(const PassCfg& cfg);

// Reduction, K-space step and the two-pass path (weiszfeld.hip).
hipError_t launch_slab_reduce(const double* slab, int nb, int64_t S, double* sums,
                              const KState* st, hipStream_t s, int problems = 1,
                              int64_t sums_ps = 0);
hipError_t launch_kspace(const KspaceArgs& a, hipStream_t s, int problems = 1);
hipError_t launch_twopass(bool init, const float* X, int64_t K, int64_t d, int64_t ldx,
                          const float* g_old, float* g_new, const float* coef, const KState* st,
                          int noise, const float* hnoise, uint64_t seed, int64_t iter,
                          int64_t col_off, double* slab, int nb, double* sums, hipStream_t s);
int twopass_blocks(int64_t K, int64_t d, int num_cu);
hipError_t launch_batched_finalize(const float* g0, const float* g1, int64_t d, int problems,
                                   const KState* st, float* out, int64_t ldo, hipStream_t s);

// Register-resident persistent kernel for small problems (resident.hip).
struct ResArgs {
  const float* X;
  int64_t K, d, ldx;
  // panels (pstride > 0): element (k, j) at X + (j >> wshift) * pstride + k * 2^wshift +
  // (j & (2^wshift - 1)); rows [K][ldx] otherwise
  int64_t pstride;
  int wshift;
  const float* guess0;
  float* out;
  int64_t maxiter;
  float tol, eps;
  int mode, has_noise;
  double P_max, noise_sd;
  uint64_t seed;
  unsigned long long* gran;  // [2][gridDim.x][2K + 2] {tag, fp32} granules (zeroed per call)
  unsigned* bar;         // [2] timeout flag, [3] check-in passed (zeroed per call)
  unsigned long long* checkin;   // [gridDim.x + 1] co-residency slots (zeroed per call)
  unsigned need;         // slots the check-in waits for (gridDim.x; + 1 forces a failure)
  // 1, or 8: the grid is 8x the working blocks and only blocks b % 8 == 0 work (logical
  // block b / 8), so that — workgroups being dispatched round-robin over the 8 XCDs — every
  // working block sits on ONE XCD and the exchange stays inside its L2 (A/B knob)
  unsigned stride;
  // 1: when the check-in finds every block on one XCD, the granules are stored so that
  // they stay in that XCD's L2 (resident.hip put_value); 0: agent-scope stores always
  int local;
  // XCD-hierarchical gather (grids beyond one XCD, stride 1): blocks b with b % 8 == x form
  // group x (the blocks dispatch places on XCD x); each block publishes to its group, the
  // group's first block (the leader) sums its members and publishes the group sum as an
  // fp32 {hi, lo} granule pair into lvl2 [2][8][2 (2K + 2)]; every block sums the 8 group
  // sums in group order.  0: the flat gather over every block.
  int hier;
  unsigned long long* lvl2;
  // split-scope exchange (stride 1, not hier): every granule also stored L2-kept into
  // granL [2][gridDim.x][2K + 2]; a reader polls its own XCD's blocks (b % 8 == its group)
  // there once the check-in confirms the group on one XCD
  int split;
  unsigned long long* granL;
  KState* st;
};
// Plan a resident launch over nch chunks: chunks per block and blocks (false: the
// grid cannot be co-resident / no kernel for the tile).
bool resident_plan(const PassCfg& cfg, int64_t nch, int num_cu, int* cpb, int* nb);
size_t resident_gran_words(int64_t K, const PassCfg& cfg, int nb);
// whether the resident kernel of this tile has exchange variant xg (1 hierarchical, 2 split)
bool resident_has_exchange(const PassCfg& cfg, int cpb, int xg);
hipError_t launch_resident(const PassCfg& cfg, int cpb, int grid, const ResArgs& a, hipStream_t s);
bool res_coop_launch();   // GMAGG_RES_COOP=1: cooperative launches (resident.hip)

// Register-resident batched kernel (resident_batched.hip, C5): NG groups of NB blocks,
// group g runs problems g, g + NG, ... each held in VGPRs for all its iterations.
struct ResBArgs {
  const float* X;         // problem p at X + p * x_ps; rows [K][ldx] or panels (pstride > 0)
  int64_t P, K, d, ldx, x_ps, pstride;
  int wshift;             // panels: W = 1 << wshift
  int prob_bytes;         // bytes of one problem's buffer (< 2^31; the loads' range)
  int nb;                 // blocks per group
  const float* guess0;
  int64_t ldg;
  float* out;
  int64_t ldo;
  int64_t maxiter;
  float tol, eps;
  int mode, has_noise;
  double P_max, noise_sd;
  uint64_t seed;          // AirComp Philox key (problem p: seed + p * kSeedStride)
  int pre_oma;            // gm2 --var: OMA pre-noise in registers, written back to X
  float oma_sd;
  uint64_t oma_seed;
  unsigned long long* gran;  // [NG][2][NB][2K + 2] {tag, fp32} granules (zeroed per call)
  unsigned* flag;         // [0] timeout flag, [2] check-in passed (zeroed per call)
  unsigned long long* checkin;   // [gridDim.x + 1] co-residency slots (zeroed per call)
  unsigned need;          // slots the check-in waits for (gridDim.x; + 1 forces a failure)
  // 1: logical block = blockIdx.x (a group's NB blocks round-robin over all 8 XCDs);
  // XCD-major: logical blocks numbered XCD by XCD (b % 8 first), so a group of NB blocks
  // spans ceil(NB / 32) + 1 XCDs instead of 8 (A/B knob)
  int xcd_major;
  // 1: groups whose blocks the check-in finds on one XCD store their granules into that
  // XCD's L2 (resident_batched.hip rb_put); the plan then gives each XCD whole groups
  int local;
  // 1 (with xcd_major): the XCD-hierarchical gather — a group's blocks gather by XCD
  // (sub-group leaders), then every block sums the <= 8 sub-group sums in lvl2
  // [NG][2][8][2 (2K + 2)] (resident_batched.hip)
  int hier;
  unsigned long long* lvl2;
  KState* st;             // [P]
};
struct RbPlan {
  int kr;                 // rows held per thread (K rounded up: 16, 32 or 52)
  int nb;                 // blocks per problem (2048 columns each)
  int ng;                 // problems in flight (groups)
  int mode;               // gm_mode (the kernel is built per mode)
};
// xcd_whole: whole groups per XCD (8 x floor(cap / 8 / nb) groups, when that is >= 8), so
// that each group's blocks share one L2 (GMAGG_RB_XCD=2)
bool rb_plan(int64_t K, int64_t d, int64_t P, int mode, int num_cu, RbPlan* plan,
             bool xcd_whole = false);
size_t rb_gran_words(int64_t K, const RbPlan& plan);
hipError_t launch_resident_batched(const RbPlan& plan, const ResBArgs& a, bool coop, hipStream_t s);

// Gram-space variant (gram.hip).  KT = K padded to 32-row tiles (0: unsupported).
// H16: scaled f16 h+m split, 3 products on v_mfma_f32_32x32x16_f16 (default);
// BF16: bf16 h+m split, 4 products on v_mfma_f32_32x32x16_bf16 (fallback when
// the f16 Gram is non-finite); F32: exact f32-input v_mfma_f32_32x32x2_f32.
enum class GramKind { F32, BF16, H16 };
struct GramGrid {
  int nb;          // blocks
  int64_t cpb;     // columns per block
  int nseg;        // fp32 partials per block
};
int gram_kt(int64_t K);
GramGrid gram_grid(int64_t d, GramKind kind, int num_cu);
size_t gram_slab_floats(int KT, const GramGrid& g);
// the f16 kernel's per-block scale exponents (written by every H16 launch_gram)
int* gram_block_exp(float* slab, int KT, const GramGrid& g);
// pstride > 0: X in the panel layout [ceil(d/W)][K][W], W = 1 << wshift (H16 only).
hipError_t launch_gram(const float* X, int64_t K, int64_t d, int64_t ldx, const float* p,
                       GramKind kind, const GramGrid& g, float* slab, double* G, KState* st,
                       hipStream_t s, int64_t pstride = 0, int wshift = 0);
hipError_t launch_gram_check(const double* G, int KP, KState* st, hipStream_t s);
hipError_t launch_gram_verify(const double* G, int KP, int64_t K, float eps, const double* u,
                              const double* alpha, const double* Dx, double* bvec, KState* st,
                              hipStream_t s);
hipError_t launch_gram_solve(const double* G, int KP, int64_t K, int64_t maxiter, float tol,
                             float eps, double* alpha, double* u, float* coef, KState* st,
                             hipStream_t s);

// Other aggregators (coordinate.hip).
// ws > 0: X in the panel layout [ceil(d/W)][K][W], W = 2^ws, ldx = the panel stride.
hipError_t launch_col_mean(const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                           hipStream_t s, int ws = 0);
hipError_t launch_col_select(const float* X, int64_t K, int64_t d, int64_t ldx, int mode,
                             int64_t b, float* out, hipStream_t s, int ws = 0);
// getVarience (M:127-129): one streaming pass, part[nb] fp64 block partials.
int honest_var_blocks(int64_t d, int num_cu);
hipError_t launch_honest_var(const float* X, int64_t H, int64_t d, int64_t ldx, int wshift,
                             int nb, double* part, float* out, hipStream_t s);
// Krum: D [K][K] fp64, part [krum_slices(K, d)][K][K] fp64, score [K] fp64.
int64_t krum_slices(int64_t K, int64_t d);
hipError_t launch_krum(const float* X, int64_t K, int64_t d, int64_t ldx, int64_t kk, double* D,
                       double* part, double* score, float* out, int64_t* index, hipStream_t s,
                       int ws = 0);
// Krum through the Gram (round 5): bounds + candidates from G [KP][KP] (lb, ub [K]; cand
// [2 + maxc] int64: count, -1 (a bound not finite) or -2 (more than maxc), the indices, then
// the row of the smallest upper bound), the candidates' exact rows (at most
// krum_refine_max() per launch; part [krum_slices][m][K], Dc [m][K], score [m]), the pick.
hipError_t launch_copy_row_k(const float* X, int64_t d, int64_t ldx, int ws, int64_t k, float* out,
                             hipStream_t s);
hipError_t launch_krum_gram_select(const double* G, int KP, int64_t K, int64_t kk, double epsg,
                                   const int* bexp, int nb, int64_t d, double* lb, double* ub,
                                   int64_t maxc, int64_t* cand, hipStream_t s);
int krum_refine_max();
hipError_t launch_krum_refine(const float* X, int64_t K, int64_t d, int64_t ldx, int ws,
                              const int64_t* cidx, int m, int64_t kk, double* part, double* Dc,
                              double* score, hipStream_t s);
hipError_t launch_krum_pick(const double* score, const int64_t* cidx, int64_t m, const float* X,
                            int64_t d, int64_t ldx, int ws, int64_t* index, float* out,
                            hipStream_t s);

// The clients' local SGD chain of one federated step (clients.hip).
struct ClientChainArgs {
  const float* data;      // training set [n][ldd] fp32 (row = one flattened sample)
  int64_t ldd;
  const int64_t* labels;  // [n]
  int64_t F, C;           // features, classes (the MLP's weight is [C][F])
  const int* idx;         // [K][B] dataset rows of each client's batch
  int64_t K, B, honest;
  int attack;             // 0 none / weightflip, 1 classflip, 2 dataflip
  float gamma, wd;
  float* W;               // [C][F], updated in place (the model's weight)
  float* b;               // [C]
  float* X;               // client matrix: rows [K][ldx] or panels
  int64_t ldx;            // rows: row stride
  int64_t pstride;        // > 0: panels, elements between panels (panel width 1 << wshift)
  int wshift;
  int stage;              // (set by launch_client_chain) the batch tile staged in LDS
};
bool client_chain_supported(int64_t F, int64_t C, int64_t B);
hipError_t launch_client_chain(const ClientChainArgs& a, hipStream_t s);

// OMA / synthetic fills (oma.hip).
hipError_t launch_oma_apply(float* X, int64_t K, int64_t d, int64_t ldx, const float* hr,
                            const float* hi, const float* nr, const float* ni, hipStream_t s);
hipError_t launch_rows_to_panels(const float* X, int64_t K, int64_t d, int64_t ldx, float* P,
                                 int64_t W, int64_t pstride, hipStream_t s);
hipError_t launch_oma_philox(float* X, int64_t K, int64_t d, int64_t ldx, int64_t d_total,
                             int64_t col_off, float sd, uint64_t seed, hipStream_t s,
                             int wshift = 0, int64_t problems = 1, int64_t pstride = 0);
hipError_t launch_fill_clients(float* X, int64_t K, int64_t d, int64_t ldx, int64_t B,
                               float mu_h, float sd_h, float mu_b, float sd_b, int64_t d_total,
                               int64_t col_off, uint64_t seed, hipStream_t s);
hipError_t launch_fill_normal(float* v, int64_t n, float mu, float sd, int64_t off,
                              uint64_t seed, hipStream_t s);

}  // namespace gmk
