/*
 * qsc.h — C ABI of libqsc_hip.so, the MI355X (gfx950) hot path of the one-bit / quantized
 * maximum-likelihood tensor factorisation of shresthasagar/quantized_spectrum_cartography.
 *
 * The reference has no native boundary: its hot path is module-level Python on torch CPU
 * tensors (qmc/quantization_model.py, qmc/quantization_model_log.py) driven by the alternating
 * solver in qmc/qmc.ipynb cell 1 (raw-JSON lines :559-645).  Each entry point below names the
 * reference function it replaces (file:line).  The Python package
 * quantized_spectrum_cartography_amd binds these symbols with ctypes.
 *
 * Conventions
 *   - every pointer argument is DEVICE memory owned by the caller (contiguous, naturally
 *     aligned), except arguments documented as host pointers (qsc_model*, qsc_obs_desc*);
 *   - the library never allocates device memory: callers size workspaces with the
 *     *_workspace_bytes() queries;
 *   - every call is asynchronous on the given hipStream_t (passed as void*), except the two
 *     calls documented as synchronous (qsc_obs_layout, qsc_device_check);
 *   - return value: 0 on success, QSC_EINVAL on a bad argument, otherwise a hipError_t.
 *
 * Tensor layouts (fp32 unless stated; "pixel" p = i*J + j, P = I*J):
 *   S   [R][P]        emitter spatial loss fields   (reference S: (R,1,I,J))
 *   C   [R][K]        emitter power spectra         (reference C: (R,K))
 *   T   [K][P]        radio map T = sum_r S_r (x) c_r (reference get_tensor output (K,I,J))
 *   Y   [K][P] int64  bin indices                   (reference quantize output)
 *   codes [K][P] u8   Y with the sampling mask folded in: 0xFF = unobserved
 */
#ifndef QSC_H_
#define QSC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QSC_API __attribute__((visibility("default")))

#define QSC_OK 0
#define QSC_EINVAL 100000
#define QSC_EUNSUPPORTED 100001 /* configuration this library build does not run */
#define QSC_MAX_BOUNDS 256 /* nbins <= 255: code 0xFF is the "unobserved" sentinel */
#define QSC_MAX_R 16       /* rank bound of the fused passes */
#define QSC_UNOBSERVED 0xFF

/* Probit observation model, host struct passed by pointer.
 *   reference: F_probit qmc/quantization_model.py:57-61 (constant 1.414213, kept verbatim);
 *              prob_probit qmc/quantization_model.py:22-39 (linear: b[0]=-1e5, b[-1]=1e5 clamp)
 *              and qmc/quantization_model_log.py:23-41 (log model: no clamp);
 *              quantize qmc/quantization_model.py:8-20 / _log.py:9-21 (b[-1]=inf).
 * sigma and offset are doubles because the reference passes Python floats: the library forms
 * fp32(sigma*1.414213) and fp32(offset) exactly as torch does for a tensor-scalar op. */
typedef struct qsc_model {
  int32_t nbounds;   /* number of bin boundaries = nbins + 1, 2..QSC_MAX_BOUNDS */
  int32_t log_model; /* 0: linear model, 1: log-domain model x = log(t + offset) */
  double sigma;      /* probit noise standard deviation */
  double offset;     /* log-model offset (ignored when log_model == 0) */
  float bounds[QSC_MAX_BOUNDS]; /* bin boundaries as the caller gives them (unclamped) */
  int32_t loss;      /* QSC_LOSS_PROBIT (0) or QSC_LOSS_SQUARED (1), see below */
  int32_t reserved_;
} qsc_model;
/* loss of the fused passes (qsc_spass / qsc_cpass):
 *   QSC_LOSS_PROBIT:  -sum_obs log P(y | x)                        qmc/qmc.ipynb :572, :631
 *   QSC_LOSS_SQUARED:  sum_obs (x - Obs)^2, Obs = (b[y] + b[y+1]) / 2 on the raw edges
 *                      (get_quantized_obs_from_ordinal, qmc/quantization_model_log.py:43-51):
 *                      the Euclidean "DowJons" criterion ||Wx (T_hat - Obs)||_F^2 of
 *                      qmc/qmc_dowjons.ipynb :142, :160 (sigma is unused).
 * with x = t (linear) or log(t + offset) (log model); the state's nll_* fields then hold the
 * squared-loss sums. */
#define QSC_LOSS_PROBIT 0
#define QSC_LOSS_SQUARED 1

/* Adam hyper-parameters (torch.optim.Adam defaults: betas (0.9, 0.999), eps 1e-8).  The
 * per-step bias corrections are computed on the device from the step counters held in the
 * solver state, so one captured hipGraph can be replayed for every iteration. */
typedef struct qsc_adam {
  double lr; /* doubles: torch forms 1 - beta^step and lr / bc1 in Python floats */
  double beta1;
  double beta2;
  double eps;
  int32_t project_nonneg; /* apply x[x<0] = 0 after the step (qmc/qmc.ipynb :579) */
  int32_t pad_;
} qsc_adam;

/* Device-resident solver scalars (one struct per solve, caller-allocated device memory,
 * initialised by qsc_state_init).  Kernels read and write it; the host reads it back only
 * when it wants the cost history.  Book-keeping protocol (no extra launches per iteration):
 * every block of a kernel reads the counters it needs at its start; the one-thread updates
 * are deferred to the NEXT kernel of the other block type through `pending`:
 *   cfinish (mode 1) sets QSC_PEND_C; the next qsc_spass applies step_c += 1;
 *   qsc_spass sets QSC_PEND_SNLL (and qsc_spass mode 1 / qsc_supdate set QSC_PEND_SUPD);
 *   the next qsc_cfinish (or qsc_state_flush) reduces the S-side partials into nll_s /
 *   normsq_s, applies step_s += 1 and appends the history row of that iteration. */
#define QSC_PEND_C 1
#define QSC_PEND_SNLL 2
#define QSC_PEND_SUPD 4
typedef struct qsc_state {
  int32_t step_c;   /* Adam steps taken on C */
  int32_t step_s;   /* Adam steps taken on S */
  int32_t iter;     /* S-passes issued (outer iterations) */
  int32_t pending;  /* QSC_PEND_* flags, see above */
  float normsq_s;   /* ||S||_F^2 of the current S */
  float normsq_c;   /* ||C||_F^2 of C before the last C update */
  float nll_c;      /* NLL of the last C-pass   (-sum Wx log P, qmc/qmc.ipynb :572) */
  float nll_s;      /* NLL of the last S-pass */
  float normsq_s_prev; /* ||S||^2 the last S-pass was evaluated with */
  int32_t fused_fault; /* reserved, 0 (the fault word of round 4-5's one-launch forms, which
                          were measured slower than the launch pairs and removed) */
  uint64_t fin_ticket; /* reserved, 0 */
  float reserved[4];
} qsc_state;

/* Packed observation layout, produced by qsc_obs_layout (host struct).
 * Positions q in 0..Pp-1 are pixels re-ordered by observation count (perm[q] = pixel).
 *  S-format ("pixel slices"): for slice s (QSC_SLICE = 32 positions), position l in the slice,
 *     entry j < s_width[s]:
 *     idx = s_off[s] + (j/4)*128 + l*4 + (j%4);  value = k | code << KBITS  (code PAD = pad)
 *     (the S-pass gives each pixel two lanes, which take alternate 4-entry chunks) */
#define QSC_SLICE 32
/* Both entry arrays end with QSC_ENTRY_TAIL pad entries (counted in s_entries / c_entries) so
 * that the passes may issue their read-ahead loads without bounds branches. */
#define QSC_ENTRY_TAIL 256
/*
 *  C-format ("frequency slices" per pixel tile): tile t (PT positions), k-slice ks (64 lanes),
 *     lane l walks bin k = c_kmap[(t*nks+ks)*64 + l], entry j < c_width[t*nks+ks]:
 *     idx = c_off[t*nks+ks] + (j/4)*256 + l*4 + (j%4);  value = qlocal | code << QBITS
 *     c_kmap: per tile, the bins 0..64*nks-1 (those >= K are empty padding bins) ordered by
 *     their observation count in the tile, descending (ties: lower k first).  A wave walks its
 *     64 lists in lockstep, padded to the longest; count-sorted slices keep that padding small
 *     (C3: 24 % of the entries with k = 64*ks + l, a few % sorted).
 *     Tile rows are whole S-format slices dealt in snake order, so that every tile holds the
 *     same mix of dense and sparse positions (positions are count-sorted): row qlocal of tile t
 *     is position  g*QSC_SLICE + qlocal%QSC_SLICE,  g = i*ntiles + (i odd ? ntiles-1-t : t),
 *     i = qlocal/QSC_SLICE.
 *  narrow (wide == 0): uint16 entries, KBITS = QBITS = 12, code PAD = 15 (K, PT <= 4096, nbins <= 15)
 *  wide   (wide == 1): uint32 entries, KBITS = QBITS = 24, code PAD = 255
 *  Signed-row entries (rowfmt == 1; one-bit linear model, narrow only, set by the caller between
 *  qsc_obs_layout and qsc_obs_fill when qsc_obs_signed_rows_ok): the value is the row of the
 *  pass's LDS table directly -- with  Ko = round_up(K, 16), Qo = round_up(PT, 16):
 *  S-format  k + (code == 1 ? Ko : 0),  pads 2Ko + r;  C-format  qlocal + (code == 1 ? Qo : 0),
 *  pads 2Qo + r  (r in 0..15).  The passes stage each factor row twice, as [+row, +thr'] and
 *  [-row, -thr'] (thr' the scaled threshold), plus 16 neutral pad rows, so an entry's code is
 *  applied by the gather itself (z of code 1 is -z of code 0, exactly).
 *  List order: qsc_obs_fill writes each list in ascending k / qlocal order with its pads last;
 *  qsc_obs_schedule may then permute every list (and choose its pads' rows r) so that the lanes
 *  of each 16-lane ds_read_b128 group read rows of distinct residues mod 16 at every slot --
 *  bank-conflict-free gathers.  The passes accept either order (a list's order only changes the
 *  order its gradient terms are summed in). */
typedef struct qsc_obs_desc {
  int32_t K;      /* frequency bins in this (local) slab */
  int32_t P;      /* pixels I*J */
  int32_t Pp;     /* P rounded up to PT */
  int32_t PT;     /* C-pass pixel tile (positions), multiple of 64, <= 4096 when narrow */
  int32_t ntiles; /* Pp / PT */
  int32_t nks;    /* ceil(K / 64) */
  int32_t wide;   /* entry width selector, see above */
  int32_t nbins;  /* number of bins (codes 0..nbins-1) */
  int64_t nnz;    /* observed entries */
  int64_t s_entries; /* S-format entries incl. padding */
  int64_t c_entries; /* C-format entries incl. padding */
  int32_t rowfmt; /* 0: code-field entries; 1: signed-row entries (see above) */
  int32_t reserved_;
} qsc_obs_desc;

/* ---------------------------------------------------------------------------------------
 * library / device
 * ------------------------------------------------------------------------------------- */
QSC_API int qsc_version(void);
/* rank padding of the position-order factor layout: 4, 8 or 16 (R <= QSC_MAX_R), else 0 */
QSC_API int qsc_rank_pad(int32_t R);
QSC_API const char* qsc_error_string(int code);
/* synchronous: returns 0 if device `dev` is a gfx950 the code objects can run on */
QSC_API int qsc_device_check(int dev);

/* ---------------------------------------------------------------------------------------
 * elementwise model ops
 * ------------------------------------------------------------------------------------- */
/* quantize: qmc/quantization_model.py:8-20 (linear), qmc/quantization_model_log.py:9-21 (log).
 * noise = torch.randn(X.shape) drawn by the caller (host RNG, as in the reference);
 * x = X + noise*fp32(sigma) (linear) or log(X + offset) + noise*fp32(sigma) (log);
 * Y = i for b[i] < x <= b[i+1] (i >= 1, b[-1] = +inf), else 0.                             */
QSC_API int qsc_quantize(const float* X, const float* noise, int64_t n, const qsc_model* m,
                         int64_t* Y, void* stream);
/* bin step of quantize alone: Y = i for b[i] < x <= b[i+1] (i >= 1, b[-1] = +inf), else 0, for
 * observations x already formed by the caller.  The log model's x = log(X + offset) +
 * randn*std (qmc/quantization_model_log.py:14) is formed on the host with torch's own CPU log,
 * so that Y is bit-identical to the reference's (ocml logf and ATen's vectorised log differ by
 * an ulp on some inputs); the binning loop (qml:15-20) runs here.                            */
QSC_API int qsc_bin_codes(const float* x, int64_t n, const qsc_model* m, int64_t* Y,
                          void* stream);
/* prob_probit: qmc/quantization_model.py:22-39, qmc/quantization_model_log.py:23-41.
 * P = F(b[Y+1] - Xhat) - F(b[Y] - Xhat), F(y) = 0.5*(1 + erf(y / fp32(sigma*1.414213))). */
QSC_API int qsc_prob_probit(const int64_t* Y, const float* Xhat, int64_t n, const qsc_model* m,
                            float* P, void* stream);
/* vector-Jacobian product of prob_probit w.r.t. Xhat: gX = gP * dP/dXhat */
QSC_API int qsc_prob_probit_bwd(const int64_t* Y, const float* Xhat, const float* gP, int64_t n,
                                const qsc_model* m, float* gX, void* stream);
/* F_probit: qmc/quantization_model.py:57-61 */
QSC_API int qsc_f_probit(const float* y, int64_t n, double sigma, float* out, void* stream);
/* mid-bin values: get_quantized_obs_from_ordinal, qmc/quantization_model_log.py:43-51 */
QSC_API int qsc_obs_from_ordinal(const int64_t* Y, int64_t n, const qsc_model* m, float* out,
                                 void* stream);
/* fold the Bernoulli sampling mask Wx (qmc/qmc.ipynb :493) into uint8 codes:
 * codes = (Wx == 0) ? 0xFF : Y.  Wx may be NULL (all observed).  Entries with Y outside
 * [0, nbins) are counted into *bad (device int32, caller zeroes it). */
QSC_API int qsc_pack_codes(const int64_t* Y, const float* Wx, int64_t n, int32_t nbins,
                           uint8_t* codes, int32_t* bad, void* stream);

/* ---------------------------------------------------------------------------------------
 * reconstruction T = sum_r S_r (x) c_r
 *   reference: outer qmc/quantization_model.py:70-77, get_tensor :79-86
 *   (qmc/quantization_model_log.py:80-96).  The r-sum is accumulated in the reference's
 *   order with separate fp32 multiply and add, so T is bit-identical to get_tensor.
 * ------------------------------------------------------------------------------------- */
QSC_API int qsc_reconstruct(const float* S, const float* C, int32_t R, int32_t P, int32_t K,
                            float* T, void* stream);
/* backward of get_tensor: dS[r][p] = sum_k gT[k][p] C[r][k], dC[r][k] = sum_p gT[k][p] S[r][p].
 * Either output may be NULL.  Deterministic (fixed-order partial sums in ws). */
QSC_API size_t qsc_reconstruct_bwd_workspace_bytes(int32_t R, int32_t P, int32_t K);
QSC_API int qsc_reconstruct_bwd(const float* gT, const float* S, const float* C, int32_t R,
                                int32_t P, int32_t K, float* dS, float* dC, void* ws,
                                size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * reductions: NMSE qmc/quantization_model.py:88-92, NMSE_LOG qmc/quantization_model_log.py:104-111
 * out2[0] = sum (f(a) - f(b))^2, out2[1] = sum f(b)^2 (fp64, device), f = identity or
 * log(. + fp32(offset)) when use_log.  a == NULL means a = reconstruct(S, C) computed on the fly
 * (fused: the map is never materialised).
 * ------------------------------------------------------------------------------------- */
QSC_API size_t qsc_reduce_workspace_bytes(int64_t n);
QSC_API int qsc_diff_sumsq(const float* a, const float* b, int64_t n, int32_t use_log,
                           double offset, double* out2, void* ws, size_t ws_bytes, void* stream);
QSC_API int qsc_map_diff_sumsq(const float* S, const float* C, const float* Ttrue, int32_t R,
                               int32_t P, int32_t K, int32_t use_log, double offset,
                               double* out2, void* ws, size_t ws_bytes, void* stream);
/* the solver's NMSE history inside the iteration sequence (NMSE(get_tensor(S, C), T_true) after
 * every S-step, qmc/qmc.ipynb :582, :637): with the state's iteration counter it = st->iter,
 * when it % every == 0 writes hist[2*(it/every - 1) + {0, 1}] = {sum (T_hat - T)^2, sum T^2}
 * (slots < cap), otherwise does nothing -- so it can be captured into every iteration of a
 * replayed hipGraph.  S_pos is the passes' position-order S [Pp][RP]; iperm[p] = the position
 * of pixel p (the inverse of qsc_obs_order's perm). */
QSC_API int qsc_map_nmse_track(const float* S_pos, const int32_t* iperm, int32_t RP,
                               const float* C, const float* Ttrue, int32_t R, int32_t P,
                               int32_t K, int32_t use_log, double offset, const qsc_state* st,
                               int32_t every, double* hist, int32_t cap, void* ws,
                               size_t ws_bytes, void* stream);
/* out[0] = sum x^2 (fp32 result, fixed order) */
QSC_API int qsc_sumsq(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                      void* stream);

/* ---------------------------------------------------------------------------------------
 * observation packing (one-time setup of a solve): dense codes -> sliced sparse formats.
 * The reference evaluates every (k,p) entry and multiplies unobserved ones by Wx = 0
 * (qmc/qmc.ipynb :572); the build reads only observed entries.
 * ------------------------------------------------------------------------------------- */
/* cnt[p] = number of observed k for pixel p (async) */
QSC_API int qsc_obs_count(const uint8_t* codes, int32_t K, int32_t P, int32_t* cnt, void* stream);
/* perm[q] = pixels sorted by cnt descending, stable; positions P <= q < Pp are padding (-1).
 * Pp = P rounded up to the C-pass tile PT (a multiple of 64). */
QSC_API size_t qsc_obs_order_workspace_bytes(int32_t P);
QSC_API int qsc_obs_order(const int32_t* cnt, int32_t P, int32_t Pp, int32_t* perm, void* ws,
                          size_t ws_bytes, void* stream);
/* SYNCHRONOUS: computes slice widths/offsets of both formats and the C-format bin order, and
 * fills *desc.  s_width[Pp/QSC_SLICE], s_off[Pp/QSC_SLICE + 1], c_width[ntiles*nks],
 * c_off[ntiles*nks + 1], c_kmap[ntiles*nks*64]. */
QSC_API size_t qsc_obs_layout_workspace_bytes(int32_t K, int32_t P, int32_t PT);
QSC_API int qsc_obs_layout(const uint8_t* codes, int32_t K, int32_t P, int32_t PT, int32_t nbins,
                           const int32_t* perm, const int32_t* cnt, int32_t* s_width,
                           int64_t* s_off, int32_t* c_width, int64_t* c_off, int32_t* c_kmap,
                           void* ws, size_t ws_bytes, qsc_obs_desc* desc, void* stream);
/* 1 if the signed-row entry format (rowfmt = 1) applies to this layout at rank R under model m:
 * the one-bit linear model (saturated outer edges, probit loss), narrow entries, and the doubled
 * LDS tables of every pass fit.  Passes given a rowfmt = 1 layout they cannot run return
 * QSC_EINVAL. */
QSC_API int qsc_obs_signed_rows_ok(const qsc_obs_desc* desc, int32_t R, const qsc_model* m);
QSC_API int qsc_obs_fill(const uint8_t* codes, const qsc_obs_desc* desc, const int32_t* perm,
                         const int32_t* s_width, const int64_t* s_off, const int32_t* c_width,
                         const int64_t* c_off, const int32_t* c_kmap, void* s_entries,
                         void* c_entries, void* stream);
/* Bank-conflict-free list order (qsc_sched.cuh): re-orders the filled entries of both formats in
 * place, per 16-lane group of a slice / (tile, k-slice) block, as an edge colouring of lanes x
 * row residues (each slot holds each residue ceil(count / W) times at most, once whenever the
 * group has <= W entries of that residue).  Blocks with lists longer than 256 keep their order.
 * SYNCHRONOUS (reads the longest list width); run once per packing, after qsc_obs_fill. */
QSC_API size_t qsc_obs_schedule_workspace_bytes(const qsc_obs_desc* desc);
QSC_API int qsc_obs_schedule(const qsc_obs_desc* desc, const int32_t* s_width,
                             const int64_t* s_off, const int32_t* c_width, const int64_t* c_off,
                             void* s_entries, void* c_entries, void* ws, size_t ws_bytes,
                             void* stream);
/* Host (CPU) form of one group's schedule, the same code as the device pass (tests / tools):
 * in/out are 16 lists of W uint32 entry values, lane-major; rowfmt/rows/wide describe the
 * entry values as in qsc_obs_desc (rows = K for S-format lists, PT for C-format lists).
 * Returns 0, or 1 when the group was copied unchanged (W > 256). */
QSC_API int qsc_sched_lists_host(const uint32_t* in, uint32_t* out, int32_t W, int32_t rowfmt,
                                 int32_t rows, int32_t wide);
/* gather/scatter between natural pixel order [R][P] and position order [Pp][RP]
 * (RP = qsc_rank_pad(R); rows R..RP-1 and positions of no pixel are zero-filled / ignored) */
QSC_API int qsc_perm_gather(const float* nat, const int32_t* perm, int32_t R, int32_t P,
                            int32_t Pp, float* pos, void* stream);
QSC_API int qsc_perm_scatter(const float* pos, const int32_t* perm, int32_t R, int32_t P,
                             int32_t Pp, float* nat, void* stream);

/* ---------------------------------------------------------------------------------------
 * fused likelihood + gradient passes (the hot path)
 *   per observed entry e=(k,p):  t = sum_r S[r,p] C[r,k]  (reference order),
 *   x = t (linear) or log(t + offset), P = prob_probit, nll -= log P,
 *   g = (exp(-u^2) - exp(-w^2)) / (a sqrt(pi) P) * (log ? 1/(t+offset) : 1)
 *   dS[r,p] = sum_k g C[r,k], dC[r,k] = sum_p g S[r,p]
 *   (replaces get_tensor -> log -> prob_probit -> -sum(Wx log P) -> autograd backward,
 *    qmc/qmc.ipynb :566-575 and :626-633)
 * S, mS, vS, dS are in position order [Pp][RP] (pixel-major: a position's RP = qsc_rank_pad(R)
 * values are one 16/32/64-byte row, rows r >= R zero); C, mC, vC in [R][K].
 * ------------------------------------------------------------------------------------- */
/* Pass workspace: zero it once before its first use (the S-pass keeps a slice scheduler in it
 * and leaves it zero on exit); one workspace serves one stream at a time. */
QSC_API size_t qsc_pass_workspace_bytes(const qsc_obs_desc* d, int32_t R);
/* zero the state; normsq_s = ||S||^2 of the initial S ([Pp][RP] position order; nullable: 0) */
QSC_API int qsc_state_init(qsc_state* st, const float* S, int32_t R, int32_t Pp, void* ws,
                           size_t ws_bytes, void* stream);
/* S-pass.  mode 0: write dS (NLL gradient only, no regulariser) — used by the generator/DIP
 * solvers and K-slab sharding; mode 1: fused S-step — dS + lambda_s*S/||S|| then Adam on S
 * (S, mS, vS updated in place).  Writes per-slice partials into ws (see qsc_state). */
QSC_API int qsc_spass(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                      const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                      const float* C, int32_t mode, float* dS, float* mS, float* vS,
                      const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                      size_t ws_bytes, void* stream);
/* K-slab S-pass (north-star sharding; the gradient half of the S-step, qmc/qmc.ipynb :626-633,
 * over this rank's bins): qsc_spass mode 0 with dS written in the reduce-scatter layout of
 * nranks chunks of chunk_slices position slices, each followed by ONE extra slice
 * (dS_rs[nranks][chunk_slices + 1][QSC_SLICE][RP]), and ||C_slab||^2 of the C it read stored in
 * element 0 of every chunk's extra slice -- so the reduce-scatter of dS_rs hands every rank the
 * summed gradient of its rows AND the global ||C||^2 the next C-step's non-squared regulariser
 * needs (no separate all-reduce).  Other extra-slice elements are left untouched (keep them 0).
 * Needs chunk_slices * nranks >= Pp / QSC_SLICE. */
QSC_API int qsc_spass_kslab(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                            const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                            const float* C, float* dS_rs, int32_t chunk_slices, int32_t nranks,
                            qsc_state* st, void* ws, size_t ws_bytes, void* stream);
/* C-pass: per-tile partial dC slab + NLL partials into ws. */
QSC_API int qsc_cpass(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                      const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m, int32_t R,
                      const float* S, const float* C, void* ws, size_t ws_bytes, void* stream);
/* Fused S-step + next C-pass (free-S solver, Adam on S): one launch equal to qsc_spass(mode 1)
 * followed by qsc_cpass at the updated S -- same partials, same state protocol -- so a solver
 * runs  cpass, cfinish, (scpass, cfinish) x (n-1), spass  for n outer iterations
 * (qmc/qmc.ipynb :562-634).  One workgroup per C-pass pixel tile: the tile's S-step results
 * feed its C-pass through LDS.  Available when qsc_scpass_supported(d, R). */
QSC_API int qsc_scpass_supported(const qsc_obs_desc* d, int32_t R);
QSC_API int qsc_scpass(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                       const int64_t* s_off, const void* c_entries, const int32_t* c_width,
                       const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m,
                       int32_t R, float* S,
                       const float* C, float* mS, float* vS, const qsc_adam* adam,
                       float lambda_s, qsc_state* st, void* ws, size_t ws_bytes, void* stream);
/* reduce the C-pass slab (fixed order).  mode 0: write dC (NLL gradient only); mode 1: fused
 * C-step: dC + lambda_c*C/||C||, Adam on C, projection; mode 2 (IJ-slab sharding): as mode 0 and
 * dC[R*K] (dC holds R*K + 1 floats) receives this shard's ||S||^2 after the S-pass partials are
 * settled, so one all-reduce carries both.  Block 0 also records nll_c / normsq_c and settles a
 * pending S-pass (see qsc_state), appending history row [nll_c, nll_s, normsq_c, normsq_s] of
 * each completed iteration to hist (nullable).
 * normsq_c_ext (device, nullable): global ||C||^2 supplied by the caller (K-slab sharding). */
QSC_API int qsc_cfinish(const qsc_obs_desc* d, int32_t R, float* C, int32_t mode, float* dC,
                        float* mC, float* vC, const qsc_adam* adam, float lambda_c,
                        const float* normsq_c_ext, qsc_state* st, float* hist,
                        int32_t hist_cap, void* ws, size_t ws_bytes, void* stream);
/* C update from an externally reduced gradient g [R][K] (IJ-slab sharding, after the RCCL
 * all-reduce of the shards' dC): g + lambda_c*C/||C||, Adam on C, projection, with the state
 * protocol of qsc_cfinish mode 1.  normsq_s_ext (device, nullable): the all-reduced ||S||^2,
 * stored as the regulariser norm the next qsc_spass uses.  One workgroup (R*K is small). */
QSC_API int qsc_cupdate(int32_t R, int32_t K, float* C, float* mC, float* vC, const float* g,
                        const qsc_adam* adam, float lambda_c, const float* normsq_s_ext,
                        qsc_state* st, void* stream);
/* settle everything pending in st (S-pass partials, counters, history) — one block; used at
 * the end of a solve and between passes that are not followed by a qsc_cfinish. */
QSC_API int qsc_state_flush(const qsc_obs_desc* d, int32_t R, qsc_state* st, float* hist,
                            int32_t hist_cap, void* ws, size_t ws_bytes, void* stream);
/* S update from an externally reduced gradient g [Pp][RP] (K-slab sharding, after the RCCL
 * all-reduce of the partial dS): g + lambda_s*S/||S||, Adam on S, ||S_new||^2 partials, with
 * the same state protocol as the fused qsc_spass mode 1. */
QSC_API int qsc_supdate(const qsc_obs_desc* d, int32_t R, float* S, float* mS, float* vS,
                        const float* g, const qsc_adam* adam, float lambda_s, qsc_state* st,
                        void* ws, size_t ws_bytes, void* stream);
/* K-slab S update of this rank's shard (reduce-scatter of the partial dS ->
 * Adam on the owned 1/N of S -> all-gather): the slices [s0, s1) of S, mS, vS are updated from
 * g_own, the shard's reduce-scattered gradient ((s1-s0)*QSC_SLICE rows of RP floats, slice s0
 * first), exactly as qsc_supdate updates them; other slices are untouched.  Same state
 * protocol (the per-slice ||S_new||^2 partials of the shard; see qsc_slice_nsq). */
QSC_API int qsc_supdate_slices(const qsc_obs_desc* d, int32_t R, int32_t s0, int32_t s1,
                               float* S, float* mS, float* vS, const float* g_own,
                               const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                               size_t ws_bytes, void* stream);
/* per-slice ||S||^2 partials of every slice of S (into the pass workspace), bit-identical to
 * those qsc_supdate / qsc_supdate_slices write for the same rows: run after the all-gather of
 * the updated shards so the pending S-update settles the global ||S_new||^2 on every rank. */
QSC_API int qsc_slice_nsq(const qsc_obs_desc* d, int32_t R, const float* S, void* ws,
                          size_t ws_bytes, void* stream);
/* qsc_cpass that also writes every position slice's ||S||^2 partial (the values qsc_slice_nsq
 * writes, bit for bit) from the S tile it stages anyway: the K-slab solver's C-pass after the
 * all-gather of S, which then needs no separate qsc_slice_nsq launch. */
QSC_API int qsc_cpass_nsq(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                          const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m,
                          int32_t R, const float* S, const float* C, void* ws, size_t ws_bytes,
                          void* stream);
/* byte offset, in the pass workspace, of the float where qsc_cpass / qsc_cpass_nsq leave ||C||^2
 * of the C they read (the fixed order of qsc_sumsq_small): a K-slab solver all-reduces it in
 * place and hands it to qsc_cfinish as normsq_c_ext.  -1 on an invalid descriptor. */
QSC_API int64_t qsc_pass_cnsq_offset(const qsc_obs_desc* d, int32_t R);
/* ||x||^2 into *out (fp32, fixed order), e.g. the local ||C_slab||^2 before an all-reduce */
QSC_API int qsc_sumsq_small(const float* x, int32_t n, float* out, void* stream);
/* Adam (torch.optim.Adam's update, bit for bit with torch 2.x's single-tensor CPU path) on a flat
 * buffer of n parameters p with moments m, v and gradient g, at step = st->iter: the S-pass
 * counter, i.e. the S-step this update belongs to -- the generator / DIP solver's step on Z or
 * the decoder weights (qmc/qmc.ipynb :634), which a captured hipGraph then replays for every
 * iteration. */
QSC_API int qsc_adam_flat(float* p, float* m, float* v, const float* g, int64_t n,
                          const qsc_adam* adam, const qsc_state* st, void* stream);
/* debug builds (QSC_DEBUG=1, _build.py --debug): the source line of the last failed bounds
 * check in the pass kernels (entry offsets, gather-table rows, lane bins; a failed check is
 * recorded and its index clamped, never trapped), 0 if none, -1 in release builds.
 * SYNCHRONOUS (device synchronise); clear != 0 resets the flag. */
QSC_API int qsc_debug_status(int32_t clear);
/* diagnostics: out[0..n) = ocml erff(x), out[n..2n) = the erf of the fused passes (erf_fast) */
QSC_API int qsc_selftest_erf(const float* x, int32_t n, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * R x R normal equations (MFMA): backup/algorithms/NMF_SPA.m:18-19 pseudo-inverse and
 * backup/algorithms/joint_opt_ae.m:404-416 regularised least squares.
 *   G[R][R] = sum_p w[p] S[r,p] S[r',p]      (w = pixel mask or NULL)     -- v_mfma_f32_16x16x4_f32
 *   B[R][K] = sum_p w[p] S[r,p] T[k,p]
 *   C = (G + lambda I)^-1 B                   (Cholesky, one workgroup)
 * ------------------------------------------------------------------------------------- */
QSC_API size_t qsc_gram_workspace_bytes(int32_t R, int32_t P, int32_t K);
QSC_API int qsc_gram(const float* S, const float* w, int32_t R, int32_t P, float* G, void* ws,
                     size_t ws_bytes, void* stream);
QSC_API int qsc_gram_rhs(const float* S, const float* T, const float* w, int32_t R, int32_t P,
                         int32_t K, float* B, void* ws, size_t ws_bytes, void* stream);
QSC_API int qsc_chol_solve(const float* G, const float* B, int32_t R, int32_t K, float lambda,
                           float* X, void* stream);

/* ---------------------------------------------------------------------------------------
 * SPA warm start and non-negative C-update.
 *   qsc_syrk:  G[K][K] = sum_p w[p] T[a,p] T[b,p]   (T row-major [K][P]; K x K Gram of the
 *              data on the f32 MFMA; deterministic)
 *   qsc_spa:   backup/algorithms/NMF_SPA.m:1-29 on Tm = T' restricted to the pixel mask w
 *              (w[p] != 0 marks an observed pixel, NULL = all): SPA (NMF_SPA.m:31-56) picks up
 *              to R frequency bins into sel[R] (-1 padded; *count = how many), then
 *              C[R][K] = rows of (inv(Sm'Sm) Sm' Tm)' after ColumnPositive, C >= 0 and
 *              unit-norm (ColumnNormalization), S[R][P] = mask * T[sel] * d (Sm' of the
 *              reference, d = the column norms removed from C).  Optional G_out[K][K] copy.
 *              K <= 4096.  Stream-ordered: *count is device memory.
 *   qsc_nnls:  backup/algorithms/joint_opt_ae.m:409-417 lsqnonneg([Q'; lambda I], [y; 0]) per
 *              bin in normal-equation form: X[:,k] = argmin_{x >= 0} ||A x - b_k||, given
 *              G = Q Q^T (R x R) and B = Q Y^T (R x K); `lambda` is added to the diagonal of G
 *              (pass the reference's lambda squared).  Lawson-Hanson active set, one thread per
 *              bin; NaN column if a passive sub-system is not positive definite.
 * ------------------------------------------------------------------------------------- */
QSC_API size_t qsc_syrk_workspace_bytes(int32_t K, int32_t P);
QSC_API int qsc_syrk(const float* T, const float* w, int32_t K, int32_t P, float* G, void* ws,
                     size_t ws_bytes, void* stream);
QSC_API size_t qsc_spa_workspace_bytes(int32_t K, int32_t P, int32_t R);
QSC_API int qsc_spa(const float* T, const float* w, int32_t K, int32_t P, int32_t R,
                    int32_t* sel, int32_t* count, float* C, float* S, float* G_out, void* ws,
                    size_t ws_bytes, void* stream);
QSC_API int qsc_nnls(const float* G, const float* B, int32_t R, int32_t K, float lambda,
                     float* X, void* stream);

/* ---------------------------------------------------------------------------------------
 * Synthetic radio maps: qmc/generate_map.m:80-113.
 *   S[r][i*J+j] = min(1, (d/d0)^-alpha[r]) * 10^(shadow[r][i*J+j]/10), d = |(j res, i res) -
 *   (loc[2r], loc[2r+1])|, then S[r] /= ||S[r]||_F (f64, fixed order; norms[r] = the norm if
 *   non-NULL) and, if db, S = 10 log10(S).  shadow: the correlated shadowing field in dB
 *   (Shadowing_data.m; drawn by circulant embedding in maps.py).  The map is then
 *   qsc_reconstruct(S, C).
 * ------------------------------------------------------------------------------------- */
QSC_API size_t qsc_map_compose_workspace_bytes(int32_t R, int32_t I, int32_t J);
QSC_API int qsc_map_compose(const float* shadow, const float* loc, const float* alpha, int32_t R,
                            int32_t I, int32_t J, float res, float d0, int32_t db, float* S,
                            float* norms, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QSC_H_ */
