// qsc_pass.hip — the fused one-bit / quantized probit likelihood + gradient passes (gfx950).
//
// Replaces, per alternating-solver iteration (qmc/qmc.ipynb cell 1, :559-634):
//   T_hat = get_tensor(S, C); T_hat = log(T_hat + offset);               (:568-571, :626-629)
//   nll = -sum(Wx * log(prob_probit(Y, T_hat, b, std)))                   (:572, :631)
//   cost = nll + lambda_c*||C|| + lambda_s*||S or Z||; cost.backward()     (:573-575, :632-633)
//   optimizer.step(); C[C<0] = 0                                          (:576, :579, :634)
// with explicit gradients (include/qsc.h) over observed entries only.
//
// Work mapping (wave64):
//   S-pass: persistent grid; a wave takes 32-pixel slices (two lanes per pixel, each walking
//           half of the pixel's observed (k, code) list, S-format); S[p,:] and dS stay in
//           registers, C[:,k] is gathered from an LDS copy of C^T; the Adam update of S is
//           fused into the epilogue (no dS round trip through HBM).
//   C-pass: a 4-wave workgroup per (pixel tile, 64-bin slice); lane = bin k walking a quarter
//           of the tile's observed (pixel, code) list for k (C-format) against the tile's S rows
//           in LDS; C[:,k] and dC[:,k] stay in registers.  Per-tile dC partials go to a slab
//           that qsc_cfinish reduces in a fixed order (bitwise deterministic; no atomics).
// The per-entry math (lik_grad2, qsc_common.cuh) is branch-free and evaluates two entries per
// packed instruction where the math allows.
#include <algorithm>

#include "qsc_common.cuh"

using namespace qsc;

#if QSC_DEBUG
namespace qsc {
__device__ int g_qsc_dbg_line = 0;  // the QSC_DCHECK flag (qsc_common.cuh)
}
#endif

namespace {

constexpr int kSBlock = 256;   // S-pass / S-update: 4 waves = 4 slices of QSC_SLICE pixels
constexpr int kSWaves = kSBlock / 64;
#ifndef QSC_CPASS_BLOCK
#define QSC_CPASS_BLOCK 512
#endif
constexpr int kCBlock = QSC_CPASS_BLOCK;  // C-pass: kCBlock/64 waves = parts of one (tile, 64-bin slice)
// C-pass tile form: a bin list is split into parts while each part keeps at least this many
// 4-entry chunks and the tile form's LDS (at the signed-row size, so that both row formats of a
// layout get the same partition) fits (tile_parts; every C-pass form and the fused launches
// share the partition).  C2: 1.5 against 3.0, 145 k -> 148 k grad-steps/s
#ifndef QSC_CPART_MIN_CHUNKS
#define QSC_CPART_MIN_CHUNKS 1.5
#endif
constexpr int kFBlock = 1024;  // C finish: 16 waves split the tile sum

// occupancy targets (waves per SIMD) that bound the register allocation of the passes; the
// rank-16 instances need twice the registers for the S/C row vectors
#ifndef QSC_SPASS_WAVES
#define QSC_SPASS_WAVES 4
#endif
// fused launch: waves that read their first slice before the staging barrier (see scfused)
#ifndef QSC_EARLY_WAVES
#define QSC_EARLY_WAVES 16
#endif
// fair wave priorities: a wave lowers its s_setprio level as it progresses (S-step: per slice;
// C-pass walks: per quarter of the unit's chunk range), so the SIMD
// arbiter, oldest-first among equal levels, keeps the waves of a SIMD abreast instead of
// finishing them one after another (the last wave of a phase otherwise runs alone,
// latency-bound: profiles/r05/stamps_simd.log).  A/B at C3: fused launch -0.5 us
// (profiles/r05/ab_fair_prio.log; a per-half-slice variant was within noise and is removed)
#ifndef QSC_FAIR_PRIO
#define QSC_FAIR_PRIO 1
#endif
__device__ __forceinline__ void prio_level(int lvl) {  // 3 = most urgent
  if (lvl >= 3)
    __builtin_amdgcn_s_setprio(3);
  else if (lvl == 2)
    __builtin_amdgcn_s_setprio(2);
  else if (lvl == 1)
    __builtin_amdgcn_s_setprio(1);
  else
    __builtin_amdgcn_s_setprio(0);
}
// fused launch: a wave's first slice lands before its second slice's reads are issued
#ifndef QSC_FIRST_WAIT
#define QSC_FIRST_WAIT 1
#endif
// software-pipelined LDS gathers in the C-pass walk (walk_groups).  (The same in the S-pass
// walk spills at the 128-VGPR budget of the fused launch and was slower: DESIGN.md 7b.)
#ifndef QSC_ROW_PF_C
#define QSC_ROW_PF_C 1
#endif
// fused launch at rank <= 8: waves per workgroup (16: 128 VGPRs each; 12: 168, 3 per SIMD --
// slower, profiles/r05/ab_twelve_waves.log, with or without a software-pipelined S-step gather,
// which is removed: at 16 waves it spills)
#ifndef QSC_FUSED_WAVES
#define QSC_FUSED_WAVES 16
#endif
// fused launch: C^T staged from 16-B reads; part-sum bins read at the start
#ifndef QSC_CT_VEC
#define QSC_CT_VEC 1
#endif
#ifndef QSC_KMAP_PF
#define QSC_KMAP_PF 1
#endif
// signed-row kinds (one-bit) never read the LDS edge table: the S-pass and fused launch skip
// its read and staging, so their staging waits for the C^T reads only
#ifndef QSC_SR_SKIP_EDGES
#define QSC_SR_SKIP_EDGES 1
#endif
// C-pass parts: part p of np walks a contiguous block of its list's chunks; every C-pass form
// uses the one partition, so their sums agree bit for bit.  (Round 3's phase split of the fused
// launch -- C-pass chunks of the first S-step round's rows walked between the S-step rounds,
// which needed strided parts -- spilled at 128 VGPRs and ran slower; removed in round 6.)
#ifndef QSC_CPASS_WAVES
#define QSC_CPASS_WAVES 4
#endif
struct PartRange {
  int j0, j1, js;  // chunks j0, j0 + js, ... < j1
};
__device__ inline PartRange part_range(int W4, int p, int np) {
  return PartRange{(W4 * p) / np, (W4 * (p + 1)) / np, 1};
}
template <int RP, int W>
struct Occ {
  static constexpr int v = (RP > 8) ? (W > 4 ? 4 : W) : W;
};
// the persistent S-pass holds two slices' inputs in registers: rank 16 gets 256 VGPRs (2 waves
// per SIMD), rank 8 fits 128 (QSC_SPASS_BPC8 = 3 resident blocks: measured fastest of 2, 3, 4)
#ifndef QSC_SPASS_BPC8
#define QSC_SPASS_BPC8 3  // resident S-pass blocks per CU at rank 8 (3 waves per SIMD)
#endif
template <int RP, int EB, int W>
struct OccS {
  static constexpr int v = (RP > 8) ? (W > 2 ? 2 : W) : (RP == 8) ? QSC_SPASS_BPC8 : W;
};

// LDS row pitch (floats) of an RP-float gathered row: 16-B aligned for ds_read_b128 and, for
// RP >= 8, not a multiple of 32 B so that random rows spread over all 64 banks
template <int RP>
struct Pitch {
  static constexpr int v = (RP == 4) ? 4 : RP + 4;
};
// Signed-row tables keep each row's signed threshold (the dot product's seed) in the row
// itself: floats RP, RP+1 = {thr~, +0}, one 8-B LDS read per entry.  (A dense column of thr~/2
// after the rows, one 4-B read with the rows' banks spread 64 ways instead of 16, measured
// slower: 31.75 vs 30.97 us for the fused launch, the extra address VALU outweighing it.)
// table pitch of a likelihood kind
template <int RP, int KIND>
struct TP {
  static constexpr int v = KIND == LIK_ONEBIT_SR ? RP + 4 : Pitch<RP>::v;
};
constexpr bool is_sr(int kind) { return kind == LIK_ONEBIT_SR; }
template <int KIND>
__device__ constexpr bool stages_edges() {
  return !(QSC_SR_SKIP_EDGES && is_sr(KIND));
}
// rows of a table: K (C^T) or PT (S tile), or sr_rows(rows) with signed rows (qsc_common.cuh)
template <int KIND>
__device__ __host__ __forceinline__ int table_rows(int rows) {
  return is_sr(KIND) ? sr_rows(rows) : rows;
}
// floats of a gather table of `rows` rows
template <int RP, int KIND>
__device__ __host__ __forceinline__ int table_floats(int rows) {
  return table_rows<KIND>(rows) * TP<RP, KIND>::v;
}
// the signed thresholds of rows i (+thr~) and sr_off(rows) + i (-thr~) of a signed-row table
template <int RP, int KIND>
__device__ __forceinline__ void put_th(float* tab, int rows, int i, float th) {
  constexpr int P = TP<RP, KIND>::v;
  *reinterpret_cast<float2*>(tab + i * P + RP) = make_float2(th, 0.0f);
  *reinterpret_cast<float2*>(tab + (sr_off(rows) + i) * P + RP) = make_float2(-th, 0.0f);
}
// row i of a gather table from 4-float groups v[0..RP): signed-row tables also get the threshold
// in float RP and the negated copy at row sr_off(rows) + i
template <int RP, int KIND>
__device__ __forceinline__ void put_row4(float* tab, int rows, int i, int r, const float4& v,
                                         float th) {
  constexpr int P = TP<RP, KIND>::v;
  *reinterpret_cast<float4*>(tab + i * P + r) = v;
  if constexpr (is_sr(KIND)) {
    *reinterpret_cast<float4*>(tab + (sr_off(rows) + i) * P + r) =
        make_float4(-v.x, -v.y, -v.z, -v.w);
    if (r == 0) put_th<RP, KIND>(tab, rows, i, th);
  }
}
// the kSrPadRows neutral pad rows 2 sr_off(rows) + r of a signed-row table ([0, kPadZ]: P == 1,
// g == 0 exactly), one per bank residue r (the scheduled pads of qsc_sched.cuh)
template <int RP, int KIND>
__device__ __forceinline__ void put_pad_row(float* tab, int rows) {
  if constexpr (is_sr(KIND)) {
    constexpr int P = TP<RP, KIND>::v;
    if (threadIdx.x < kSrPadRows) {
      float* row = tab + (2 * sr_off(rows) + (int)threadIdx.x) * P;
#pragma unroll
      for (int r = 0; r < RP; ++r) row[r] = 0.0f;
      *reinterpret_cast<float2*>(row + RP) = make_float2(kPadZ, 0.0f);
    }
  }
}

template <typename E>
struct Ent;
template <>
struct Ent<uint16_t> {
  static constexpr int kBits = 12;
  static constexpr uint32_t kMask = 0xFFF;
  static constexpr int kPad = 15;
  using V4 = uint2;     // 4 entries = 8 bytes
  using V2 = uint32_t;  // 2 entries (half a chunk: the S-pass lane's share)
  __device__ static __forceinline__ void unpack(const V4& v, uint32_t (&e)[4]) {
    e[0] = v.x & 0xFFFF;
    e[1] = v.x >> 16;
    e[2] = v.y & 0xFFFF;
    e[3] = v.y >> 16;
  }
  __device__ static __forceinline__ void unpack2(const V2& v, uint32_t (&e)[2]) {
    e[0] = v & 0xFFFF;
    e[1] = v >> 16;
  }
};
template <>
struct Ent<uint32_t> {
  static constexpr int kBits = 24;
  static constexpr uint32_t kMask = 0xFFFFFF;
  static constexpr int kPad = 255;
  using V4 = uint4;  // 4 entries = 16 bytes
  using V2 = uint2;  // 2 entries
  __device__ static __forceinline__ void unpack(const V4& v, uint32_t (&e)[4]) {
    e[0] = v.x;
    e[1] = v.y;
    e[2] = v.z;
    e[3] = v.w;
  }
  __device__ static __forceinline__ void unpack2(const V2& v, uint32_t (&e)[2]) {
    e[0] = v.x;
    e[1] = v.y;
  }
};

// Per-lane global access at byte offset `lo` (32 bits) from a wave-uniform base: the address is
// SGPR base + zero-extended VGPR offset (the global_load/store saddr form), so the per-access
// 64-bit address arithmetic stays on the scalar unit instead of costing VALU per load.
template <typename T>
__device__ __forceinline__ T ld_lane(const T* base, uint32_t lo) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + lo);
}
template <typename T>
__device__ __forceinline__ void st_lane(T* base, uint32_t lo, const T& v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + lo) = v;
}

// LDS row of RP floats as RP/2 packed pairs (16-B reads)
template <int RP>
__device__ __forceinline__ void lds_row2(const float* base, f2v (&v)[RP / 2]) {
#pragma unroll
  for (int r = 0; r < RP; r += 4) {
    const float4 x = *reinterpret_cast<const float4*>(base + r);
    v[r / 2] = f2v{x.x, x.y};
    v[r / 2 + 1] = f2v{x.z, x.w};
  }
}

// t = sum_r own[r] * o[r], accumulated pairwise in r (RP/2 packed FMAs + one add)
template <int RP>
__device__ __forceinline__ float dot2(const f2v (&own)[RP / 2], const f2v (&o)[RP / 2]) {
  f2v d = own[0] * o[0];
#pragma unroll
  for (int j = 1; j < RP / 2; ++j) d = fma2(own[j], o[j], d);
  return d.x + d.y;
}

// z0 + sum_r own[r] * o[r]: the one-bit kind's z' with its offset seeded into the first FMA
template <int RP>
__device__ __forceinline__ float dot2z(const f2v (&own)[RP / 2], const f2v (&o)[RP / 2], float z0) {
  f2v d = fma2(own[0], o[0], f2v{z0, 0.0f});
#pragma unroll
  for (int j = 1; j < RP / 2; ++j) d = fma2(own[j], o[j], d);
  // an opaque (empty) asm on the sum keeps it one v_add_f32: without it the backend turns the
  // two entries' horizontal adds into three v_mov + a v_pk_add_f32
  float r = d.x + d.y;
  asm("" : "+v"(r));
  return r;
}

// the same with the seed pair read from a signed-row table ({thr~, +0}: no register move)
template <int RP>
__device__ __forceinline__ float dot2s(const f2v (&own)[RP / 2], const f2v (&o)[RP / 2], f2v seed) {
  f2v d = fma2(own[0], o[0], seed);
#pragma unroll
  for (int j = 1; j < RP / 2; ++j) d = fma2(own[j], o[j], d);
  float r = d.x + d.y;
  asm("" : "+v"(r));
  return r;
}

// factor the register row is pre-multiplied by: linear kinds evaluate in a scaled form
// (lik_grad2): -1/a (general), -sqrt(log2 e)/a (one-bit); the log model / squared loss use t
template <int KIND, bool LOG>
__device__ __forceinline__ float own_scale_of(const Lik& lk) {
  if (LOG || KIND == LIK_SQUARED) return 1.0f;
  return (KIND == LIK_ONEBIT || KIND == LIK_ONEBIT_SR) ? -lk.ob_scale : -lk.inv_a;
}

struct Scalars {
  float coef;  // lambda / ||x||  (0 when ||x|| == 0, as torch's norm backward)
  AdamScalars as;
};

// Process one 4-entry chunk as two packed pairs: `own` is the lane's register vector (S of the
// pixel or C of the frequency bin, r-pairs), `tab` the LDS table of the other factor indexed by
// the entry's low bits.  Pad entries carry index 0 (a valid row) and code kPad; the one-bit kind
// moves them to z' = kPadZ where they contribute exactly 0, the other kinds mask them.  The NLL
// is accumulated as a pair (summed by the caller).
// the LDS rows of an entry pair (the gather half of pair_step)
// (signed-row kind: the entry IS the row, whose float RP is the signed threshold -> tha/thb)
#ifndef QSC_DIAG_NOCONF_C
#define QSC_DIAG_NOCONF_C 0
#endif
#ifndef QSC_DIAG_NOCONF_S
#define QSC_DIAG_NOCONF_S 0
#endif
// Row addresses of signed-row entries (16-bit entries: the entry IS the row index).  The walks
// unpack an entry straight to its row's LDS address with one v_mad_u32_u16 (op_sel picks the
// dword's high entry): idx * pitch + the table's address, instead of a mask / shift and a
// multiply-add per entry.  (Index form in the debug and diagnostic builds, which check or
// rewrite the indices.)
#ifndef QSC_SR_ADDR
#define QSC_SR_ADDR 1
#endif
#if QSC_SR_ADDR && !QSC_DEBUG && !QSC_DIAG_NOLDS && !QSC_DIAG_NOCONF_C && !QSC_DIAG_NOCONF_S
#define QSC_SR_ADDR_ON 1
#else
#define QSC_SR_ADDR_ON 0
#endif
typedef __attribute__((address_space(3))) const char lds_char;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lds_f4v;
typedef __attribute__((address_space(3))) const f2v lds_f2v;
template <typename E, int KIND>
__device__ constexpr bool sr_addr() {
  return QSC_SR_ADDR_ON && is_sr(KIND) && sizeof(E) == 2;
}
__device__ __forceinline__ uint32_t mad_u16_lo(uint32_t v, uint32_t pb, uint32_t off) {
  uint32_t r;
  asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(pb), "s"(off));
  return r;
}
__device__ __forceinline__ uint32_t mad_u16_hi(uint32_t v, uint32_t pb, uint32_t off) {
  uint32_t r;
  asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(v), "v"(pb), "s"(off));
  return r;
}
// a gather table's LDS address (wave-uniform)
__device__ __forceinline__ uint32_t lds_off(const float* tab) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(lds_char*)reinterpret_cast<const char*>(tab));
}
// RP floats at LDS address a as RP/2 packed pairs (lds_row2 on an LDS address)
template <int RP>
__device__ __forceinline__ void lds_row2_at(uint32_t a, f2v (&v)[RP / 2]) {
#pragma unroll
  for (int r = 0; r < RP; r += 4) {
    const f4v x = *(lds_f4v*)(uintptr_t)(a + 4 * r);
    v[r / 2] = f2v{x.x, x.y};
    v[r / 2 + 1] = f2v{x.z, x.w};
  }
}
// unpack 4 / 2 entries: indices, or (sr_addr) their rows' LDS byte addresses
template <int RP, typename E, int KIND>
__device__ __forceinline__ void ent_rows4(const typename Ent<E>::V4& v, uint32_t off,
                                          uint32_t (&e)[4]) {
  if constexpr (sr_addr<E, KIND>()) {
    constexpr uint32_t PB = TP<RP, KIND>::v * 4;
    e[0] = mad_u16_lo(v.x, PB, off);
    e[1] = mad_u16_hi(v.x, PB, off);
    e[2] = mad_u16_lo(v.y, PB, off);
    e[3] = mad_u16_hi(v.y, PB, off);
  } else {
    (void)off;
    Ent<E>::unpack(v, e);
  }
}
template <int RP, typename E, int KIND>
__device__ __forceinline__ void ent_rows2(const typename Ent<E>::V2& v, uint32_t off,
                                          uint32_t (&e)[2]) {
  if constexpr (sr_addr<E, KIND>()) {
    constexpr uint32_t PB = TP<RP, KIND>::v * 4;
    e[0] = mad_u16_lo(v, PB, off);
    e[1] = mad_u16_hi(v, PB, off);
  } else {
    (void)off;
    Ent<E>::unpack2(v, e);
  }
}

// TBL: the table gathered from, 0 = C^T (S-step), 1 = the S tile (C-pass)
template <int RP, typename E, int KIND, int TBL = 0>
__device__ __forceinline__ void pair_rows(uint32_t ea, uint32_t eb, const f2v (&own)[RP / 2],
                                          const float* __restrict__ tab, f2v (&oa)[RP / 2],
                                          f2v (&ob)[RP / 2], f2v& tha, f2v& thb, const Lik& lk) {
  using T = Ent<E>;
  constexpr int P = TP<RP, KIND>::v;
  constexpr int DG = TBL == 1 ? QSC_DIAG_NOCONF_C : QSC_DIAG_NOCONF_S;
  uint32_t ia = is_sr(KIND) ? ea : (ea & T::kMask), ib = is_sr(KIND) ? eb : (eb & T::kMask);
#if QSC_DEBUG
  {
    const uint32_t lim = (uint32_t)lk.dbg_rows[TBL];
    QSC_DCHECK(ia < lim && ib < lim);
    ia = ia < lim ? ia : 0u;
    ib = ib < lim ? ib : 0u;
  }
#endif
  if constexpr (DG != 0) {
    // diagnostic builds only (wrong values): every 16-lane group of a ds_read_b128 reads rows of
    // 16 distinct residues mod 16, i.e. conflict-free gathers (bounds the bank-conflict cost)
    ia = (ia & ~15u) | (threadIdx.x & 15u);
    ib = (ib & ~15u) | (threadIdx.x & 15u);
  }
#if QSC_DIAG_NOLDS  // diagnostic build: no gather (bounds the LDS share of the pass)
#pragma unroll
  for (int j = 0; j < RP / 2; ++j) {
    oa[j] = own[j] + splat2((float)ia);
    ob[j] = own[j] + splat2((float)ib);
  }
  tha = splat2((float)ia);
  thb = splat2((float)ib);
#else
  (void)own;
  if constexpr (sr_addr<E, KIND>()) {
    // ia, ib: the rows' LDS addresses (ent_rows4 / ent_rows2)
    (void)tab;
    (void)lk;
    lds_row2_at<RP>(ia, oa);
    lds_row2_at<RP>(ib, ob);
    tha = *(lds_f2v*)(uintptr_t)(ia + RP * 4);
    thb = *(lds_f2v*)(uintptr_t)(ib + RP * 4);
    return;
  }
  lds_row2<RP>(tab + ia * P, oa);
  lds_row2<RP>(tab + ib * P, ob);
  if constexpr (is_sr(KIND)) {
#if QSC_DIAG_SR_NOTH  // diagnostic build: no threshold read (wrong values; bounds its LDS cost)
    tha = thb = f2v{0.5f, 0.0f};
#else
    tha = *reinterpret_cast<const f2v*>(tab + ia * P + RP);
    thb = *reinterpret_cast<const f2v*>(tab + ib * P + RP);
#endif
    (void)lk;  // (the table's layout is static)
  } else {
    tha = thb = splat2(0.0f);
  }
#endif
}

// the arithmetic half of pair_step on already gathered rows oa, ob
template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void pair_math(uint32_t ea, uint32_t eb, const f2v (&own)[RP / 2],
                                          const f2v (&oa)[RP / 2], const f2v (&ob)[RP / 2],
                                          f2v tha, f2v thb,
                                          const float2* __restrict__ edges, const Lik& lk,
                                          f2v (&acc)[RP / 2], f2v& nll, f2v& pq, bool valid);

template <int RP, typename E, int KIND, bool LOG, int TBL>
__device__ __forceinline__ void pair_step(uint32_t ea, uint32_t eb, const f2v (&own)[RP / 2],
                                          const float* __restrict__ tab,
                                          const float2* __restrict__ edges, const Lik& lk,
                                          f2v (&acc)[RP / 2], f2v& nll, bool valid) {
  f2v oa[RP / 2], ob[RP / 2];
  f2v tha, thb, pq;
  pair_rows<RP, E, KIND, TBL>(ea, eb, own, tab, oa, ob, tha, thb, lk);
  pair_math<RP, E, KIND, LOG>(ea, eb, own, oa, ob, tha, thb, edges, lk, acc, nll, pq, valid);
  if constexpr (is_sr(KIND)) nll -= log2_2(pq);  // (single pair: the walks pair them up)
}

template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void pair_math(uint32_t ea, uint32_t eb, const f2v (&own)[RP / 2],
                                          const f2v (&oa)[RP / 2], const f2v (&ob)[RP / 2],
                                          f2v tha, f2v thb,
                                          const float2* __restrict__ edges, const Lik& lk,
                                          f2v (&acc)[RP / 2], f2v& nll, f2v& pq, bool valid) {
  using T = Ent<E>;
  if constexpr (is_sr(KIND)) {
    // signed rows: z~ = thr~ + own . row~ (both carry the entry's sign), no code / pad handling
    f2v t = f2v{dot2s<RP>(own, oa, tha), dot2s<RP>(own, ob, thb)};
    if (!valid) t = splat2(kPadZ);  // walk_masked's evaluations past a list end
    // P goes to the caller (pq), which takes log2 of two pairs' product: the NLL costs one
    // v_log per four entries (P >= 2^-25 or exactly 0, so four factors stay normal in fp32)
    f2v g;
#if QSC_DIAG_NOMATH
    g = t * splat2(1e-3f);
    pq = splat2(1.0f) + t * splat2(1e-30f);
#else
    onebit_sr_pg(t, lk, pq, g);
#endif
    (void)nll;
    (void)edges;
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) acc[j] = fma2(splat2(g.x), oa[j], acc[j]);
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) acc[j] = fma2(splat2(g.y), ob[j], acc[j]);
    (void)ea;
    (void)eb;
    return;
  } else {
    const int ca = (int)(ea >> T::kBits), cb = (int)(eb >> T::kBits);
    const bool pa = (ca == T::kPad) || !valid, pb = (cb == T::kPad) || !valid;
    f2v t;
    if constexpr (KIND == LIK_ONEBIT)
      t = f2v{dot2z<RP>(own, oa, lk.ob_thr), dot2z<RP>(own, ob, lk.ob_thr)};
    else
      t = f2v{dot2<RP>(own, oa), dot2<RP>(own, ob)};
    f2v log2P, g;
#if QSC_DIAG_NOMATH  // diagnostic build: no likelihood arithmetic (bounds the VALU share)
    g = t * splat2(1e-3f);
    log2P = t;
#else
    if constexpr (KIND == LIK_ONEBIT)
      lik_grad2<KIND, LOG>(t, ca, cb, pa, pb, edges, lk, log2P, g);
    else
      lik_grad2<KIND, LOG>(t, pa ? 0 : ca, pb ? 0 : cb, pa, pb, edges, lk, log2P, g);
#endif
    float ga = g.x, gb = g.y;
    if constexpr (KIND == LIK_ONEBIT) {
      nll -= log2P;  // log2 units: scaled by ln 2 later
    } else {
      ga = pa ? 0.0f : ga;
      gb = pb ? 0.0f : gb;
      nll -= f2v{pa ? 0.0f : log2P.x, pb ? 0.0f : log2P.y};
    }
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) acc[j] = fma2(splat2(ga), oa[j], acc[j]);
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) acc[j] = fma2(splat2(gb), ob[j], acc[j]);
  }
}

// one 4-entry chunk (the C-pass lane's unit) as two pairs
template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void chunk(const typename Ent<E>::V4& v, const f2v (&own)[RP / 2],
                                      const float* __restrict__ tab,
                                      const float2* __restrict__ edges, const Lik& lk,
                                      f2v (&acc)[RP / 2], f2v& nll, bool valid = true) {
  uint32_t e[4];
  ent_rows4<RP, E, KIND>(v, sr_addr<E, KIND>() ? lds_off(tab) : 0u, e);
  if constexpr (is_sr(KIND)) {
    // the software-pipelined walk's arithmetic exactly (one v_log of the chunk's four P), so
    // the C-pass NLL is the same whichever walk form evaluates a chunk
    f2v oa[RP / 2], ob[RP / 2], tha, thb, pqa, pqb;
    pair_rows<RP, E, KIND, 1>(e[0], e[1], own, tab, oa, ob, tha, thb, lk);
    pair_math<RP, E, KIND, LOG>(e[0], e[1], own, oa, ob, tha, thb, edges, lk, acc, nll, pqa,
                                valid);
    pair_rows<RP, E, KIND, 1>(e[2], e[3], own, tab, oa, ob, tha, thb, lk);
    pair_math<RP, E, KIND, LOG>(e[2], e[3], own, oa, ob, tha, thb, edges, lk, acc, nll, pqb,
                                valid);
    const f2v pp = pqa * pqb;
    nll.x -= __builtin_amdgcn_logf(pp.x * pp.y);
  } else {
    pair_step<RP, E, KIND, LOG, 1>(e[0], e[1], own, tab, edges, lk, acc, nll, valid);
    pair_step<RP, E, KIND, LOG, 1>(e[2], e[3], own, tab, edges, lk, acc, nll, valid);
  }
}

// half a chunk (the S-pass lane's unit: the pixel's two lanes split every chunk)
template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void half_chunk(const typename Ent<E>::V2& v, const f2v (&own)[RP / 2],
                                           const float* __restrict__ tab,
                                           const float2* __restrict__ edges, const Lik& lk,
                                           f2v (&acc)[RP / 2], f2v& nll) {
  uint32_t e[2];
  Ent<E>::unpack2(v, e);
  pair_step<RP, E, KIND, LOG, 0>(e[0], e[1], own, tab, edges, lk, acc, nll, true);
}

// Read-ahead of a lane list in groups of NB chunks (chunk j at src[j * row], row in V4 units).
// Loads are unconditional with the index clamped to the lane's last chunk (the entry arrays end
// with a QSC_ENTRY_TAIL pad, so even an empty list's chunk 0 is addressable): the number of
// loads in flight is static, so the compiler waits for exactly the group it consumes
// (vmcnt(NB)) instead of draining every prefetch at a branch merge.
constexpr int kGroup = 4;
constexpr int kSchedQ = 16;  // S-pass slice queues (scheduler counters), QSC_PASS workspace

template <typename V4>
__device__ __forceinline__ void load_group(const V4* __restrict__ src, uint32_t lo, int row, int jb,
                                           int js, int jlast, V4 (&b)[kGroup]) {
#pragma unroll
  for (int i = 0; i < kGroup; ++i) {
    const int j = min(jb + i * js, jlast);
    b[i] = ld_lane(src + (int64_t)j * row, lo);
  }
}

// Consume group b (chunks jb, jb+js, ..., < j1), then walk the rest of the list with the next
// group's loads issued ahead of the current group's arithmetic.
template <int RP, typename E, int KIND, bool LOG, bool PFC = (QSC_ROW_PF_C != 0)>
__device__ __forceinline__ void walk_groups(const typename Ent<E>::V4* __restrict__ src,
                                            uint32_t lo, int row, int jb, int j1, int js,
                                            typename Ent<E>::V4 (&b)[kGroup],
                                            const f2v (&own)[RP / 2],
                                            const float* __restrict__ tab,
                                            const float2* __restrict__ edges, const Lik& lk,
                                            f2v (&acc)[RP / 2], f2v& nll) {
  using V4 = typename Ent<E>::V4;
  const int jlast = max(j1 - 1, 0);
#if QSC_FAIR_PRIO
  const int jfirst = jb, jspan = max(j1 - jb, 1);
  auto fair = [&]() { prio_level(3 - min(3, (4 * (jb - jfirst)) / jspan)); };
#else
  auto fair = []() {};
#endif
  const uint32_t off = sr_addr<E, KIND>() ? lds_off(tab) : 0u;
  if constexpr (PFC) {
  // software-pipelined gather: the LDS rows of the next entry pair are read before the current
  // pair's arithmetic, so the LDS latency runs under it (the group's chunks are loaded, clamped,
  // so a prefetch past the list end reads valid rows that are never used)
  f2v ra[RP / 2], rb[RP / 2];
  f2v tra, trb;
  {
    uint32_t e[4];
    ent_rows4<RP, E, KIND>(b[0], off, e);
    pair_rows<RP, E, KIND, 1>(e[0], e[1], own, tab, ra, rb, tra, trb, lk);
  }
  for (;;) {
    fair();
    const int jn = jb + kGroup * js;
    const bool more = jn < j1;
    V4 nb[kGroup];
    load_group(src, lo, row, jn, js, jlast, nb);  // unconditional: static vmcnt accounting
#pragma unroll
    for (int i = 0; i < kGroup; ++i)
      if (jb + i * js < j1) {
        uint32_t e[4];
        ent_rows4<RP, E, KIND>(b[i], off, e);
        f2v xa[RP / 2], xb[RP / 2];
        f2v txa, txb, pqa, pqb;
        pair_rows<RP, E, KIND, 1>(e[2], e[3], own, tab, xa, xb, txa, txb, lk);
        pair_math<RP, E, KIND, LOG>(e[0], e[1], own, ra, rb, tra, trb, edges, lk, acc, nll, pqa,
                                    true);
        if (i + 1 < kGroup) {
          uint32_t f[4];
          ent_rows4<RP, E, KIND>(b[i + 1], off, f);
          pair_rows<RP, E, KIND, 1>(f[0], f[1], own, tab, ra, rb, tra, trb, lk);
        }
        pair_math<RP, E, KIND, LOG>(e[2], e[3], own, xa, xb, txa, txb, edges, lk, acc, nll, pqb,
                                    true);
        if constexpr (is_sr(KIND)) {
          const f2v pp = pqa * pqb;
          nll.x -= __builtin_amdgcn_logf(pp.x * pp.y);
        }
      }
    if (!more) break;
#pragma unroll
    for (int i = 0; i < kGroup; ++i) b[i] = nb[i];
    {
      uint32_t e[4];
      ent_rows4<RP, E, KIND>(b[0], off, e);
      pair_rows<RP, E, KIND, 1>(e[0], e[1], own, tab, ra, rb, tra, trb, lk);
    }
    jb = jn;
  }
  } else {
  for (;;) {
    fair();
    const int jn = jb + kGroup * js;
    const bool more = jn < j1;
    V4 nb[kGroup];
    load_group(src, lo, row, jn, js, jlast, nb);  // unconditional: static vmcnt accounting
#pragma unroll
    for (int i = 0; i < kGroup; ++i)
      if (jb + i * js < j1) chunk<RP, E, KIND, LOG>(b[i], own, tab, edges, lk, acc, nll);
    if (!more) break;
#pragma unroll
    for (int i = 0; i < kGroup; ++i) b[i] = nb[i];
    jb = jn;
  }
  }
}

// S-pass form: the pixel's two lanes split every 4-entry chunk (lane half h takes entries 2h,
// 2h+1 of each chunk row), so both walk the same, wave-uniform chunk range [0, j1) with one
// entry pair per chunk row -- no lane idles on an odd chunk count (C3: 12 % -> 6 % padded
// evaluations).  Group b holds chunk rows jb .. jb+kGroupS-1 (src[j * row]); the next group is
// read ahead unconditionally (clamped to the last row: static vmcnt accounting).
constexpr int kGroupS = 8;

template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void walk_halves(const typename Ent<E>::V2* __restrict__ src,
                                            uint32_t lo, int row, int j1,
                                            typename Ent<E>::V2 (&b)[kGroupS],
                                            const f2v (&own)[RP / 2],
                                            const float* __restrict__ tab,
                                            const float2* __restrict__ edges, const Lik& lk,
                                            f2v (&acc)[RP / 2], f2v& nll) {
  using V2 = typename Ent<E>::V2;
  j1 = __builtin_amdgcn_readfirstlane(j1);
  const int jlast = max(j1 - 1, 0);
  int jb = 0;
  const uint32_t off = sr_addr<E, KIND>() ? lds_off(tab) : 0u;
  for (;;) {
    const int jn = jb + kGroupS;
    const bool more = jn < j1;
    V2 nb[kGroupS];
#pragma unroll
    for (int i = 0; i < kGroupS; ++i) nb[i] = ld_lane(src + (int64_t)min(jn + i, jlast) * row, lo);
    if constexpr (is_sr(KIND)) {
      // half chunks in pairs: one v_log of the four entries' product P
#pragma unroll
      for (int i = 0; i < kGroupS; i += 2)
        if (jb + i < j1) {
          f2v pa, pb = splat2(1.0f);
          {
            uint32_t e[2];
            ent_rows2<RP, E, KIND>(b[i], off, e);
            f2v oa[RP / 2], ob[RP / 2], tha, thb;
            pair_rows<RP, E, KIND, 0>(e[0], e[1], own, tab, oa, ob, tha, thb, lk);
            pair_math<RP, E, KIND, LOG>(e[0], e[1], own, oa, ob, tha, thb, edges, lk, acc, nll,
                                        pa, true);
          }
          if (jb + i + 1 < j1) {
            uint32_t e[2];
            ent_rows2<RP, E, KIND>(b[i + 1], off, e);
            f2v oa[RP / 2], ob[RP / 2], tha, thb;
            pair_rows<RP, E, KIND, 0>(e[0], e[1], own, tab, oa, ob, tha, thb, lk);
            pair_math<RP, E, KIND, LOG>(e[0], e[1], own, oa, ob, tha, thb, edges, lk, acc, nll,
                                        pb, true);
          }
          const f2v pp = pa * pb;
          nll.x -= __builtin_amdgcn_logf(pp.x * pp.y);
        }
    } else {
#pragma unroll
      for (int i = 0; i < kGroupS; ++i)
        if (jb + i < j1) half_chunk<RP, E, KIND, LOG>(b[i], own, tab, edges, lk, acc, nll);
    }
    if (!more) break;
#pragma unroll
    for (int i = 0; i < kGroupS; ++i) b[i] = nb[i];
    jb = jn;
  }
}

// Uniform-control form of walk_groups: every chunk of a group is evaluated (a chunk past the
// lane's list end reads its clamped last chunk and is masked), so the group is one basic block
// the compiler schedules as a whole (LDS gathers of later chunks under earlier chunks' math),
// and the loop trip count depends only on wave-uniform values: `ju` is the smallest first
// chunk of the wave's lanes, `j1` the (uniform) list end.  The next group is read only when
// some lane needs it.
template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void walk_masked(const typename Ent<E>::V4* __restrict__ src,
                                            uint32_t lo, int row, int jb, int ju, int j1, int js,
                                            typename Ent<E>::V4 (&b)[kGroup],
                                            const f2v (&own)[RP / 2],
                                            const float* __restrict__ tab,
                                            const float2* __restrict__ edges, const Lik& lk,
                                            f2v (&acc)[RP / 2], f2v& nll) {
  using V4 = typename Ent<E>::V4;
  j1 = __builtin_amdgcn_readfirstlane(j1);
  ju = __builtin_amdgcn_readfirstlane(ju);
  const int jlast = max(j1 - 1, 0);
  // The last group is evaluated on a path that issues no loads, so the compiler's (path-
  // insensitive) wait-count bookkeeping sees no read pending after the walk and the caller's
  // next-slice read-ahead stays in flight through the epilogue.
  for (;;) {
    const int jn = jb + kGroup * js, jun = ju + kGroup * js;
    if (jun >= j1) {  // uniform
#pragma unroll
      for (int i = 0; i < kGroup; ++i)
        chunk<RP, E, KIND, LOG>(b[i], own, tab, edges, lk, acc, nll, jb + i * js < j1);
      break;
    }
    V4 nb[kGroup];
    load_group(src, lo, row, jn, js, jlast, nb);
#pragma unroll
    for (int i = 0; i < kGroup; ++i)
      chunk<RP, E, KIND, LOG>(b[i], own, tab, edges, lk, acc, nll, jb + i * js < j1);
#pragma unroll
    for (int i = 0; i < kGroup; ++i) b[i] = nb[i];
    jb = jn;
    ju = jun;
  }
}

// ---------------------------------------------------------------------------------------
// S-pass
// ---------------------------------------------------------------------------------------
#if QSC_DIAG_STAMPS
// diagnostic builds only: per-wave timestamps of the S-pass phases (s_memtime, shader clock)
constexpr int kStampWaves = 4096, kStamps = 32;
#endif
[[maybe_unused]] constexpr int kStampLast = 31;
#if QSC_DIAG_STAMPS
__device__ unsigned long long g_stamps[kStampWaves * kStamps];
#define STAMP(w, i)                                                                  \
  do {                                                                               \
    if ((threadIdx.x & 63) == 0 && (w) < kStampWaves && (i) < kStamps)               \
      g_stamps[(w) * kStamps + (i)] = __builtin_amdgcn_s_memtime();                  \
  } while (0)
#define RSTAMP(w, i)                                                                 \
  do {                                                                               \
    if ((threadIdx.x & 63) == 0 && (w) < kStampWaves && (i) < kStamps)               \
      g_stamps[(w) * kStamps + (i)] = __builtin_amdgcn_s_memrealtime();              \
  } while (0)
#else
#define STAMP(w, i) \
  do {              \
  } while (0)
#define RSTAMP(w, i) \
  do {               \
  } while (0)
#endif

// Sum over the 64 lanes in a fixed order without LDS traffic: xor-1/xor-2 quad permutes and
// the row half-mirror / mirror DPP moves leave every lane of a 16-lane row holding the row sum;
// the four row sums are read into scalars and added in row order.  Result uniform.
__device__ __forceinline__ float dpp_f(float x, int ctrl) {
  switch (ctrl) {  // the DPP control must be an immediate
    case 0xB1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
    case 0x4E: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));
    case 0x141: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, false));
  }
}
__device__ __forceinline__ float wave_sum_dpp(float x) {
  x += dpp_f(x, 0xB1);   // quad_perm [1,0,3,2]
  x += dpp_f(x, 0x4E);   // quad_perm [2,3,0,1]
  x += dpp_f(x, 0x141);  // row_half_mirror
  x += dpp_f(x, 0x140);  // row_mirror
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
  return ((a + b) + c) + d;
}

// The S-step epilogue's lane-pair combine: a pixel's two lanes (l, l + 32) hold partial dS rows
// x = elements 0..RH-1 and y = RH..RP-1 of the same pixel; one v_permlane32_swap exchanges x's
// upper 32 lanes with y's lower ones, so lane l < 32 gets x[l] + x[l + 32] (its half's sums) and
// lane l >= 32 y[l - 32] + y[l]: half_sum + pick of both in 2 VALU, the same sums in the same
// order.  swap_lo: the value of x (lane < 32) or of y taken from the partner lane (lane >= 32):
// the half-row selection of a row both lanes hold.
__device__ __forceinline__ float half_sum_pick(float x, float y) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_lo(float x, float y) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false,
                                                  false);
  return __uint_as_float(r[0]);
}

// ||C||^2 in one fixed order (threads 0..255 stride 256, then the block sum): shared by the
// C-pass (256-thread blocks) and qsc_cupdate (1024), so both give the same bits
__device__ __forceinline__ float cnorm_sq(const float* __restrict__ C, int n, float* sh) {
  float s2 = 0.0f;
  if (threadIdx.x < 256)
    for (int i0 = threadIdx.x; i0 < n; i0 += 8 * 256) {  // 8 reads in flight, summed in order
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = C[min(i0 + 256 * j, n - 1)];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i0 + 256 * j < n) s2 = __builtin_fmaf(v[j], v[j], s2);
    }
  return block_sum(s2, sh);
}

// N consecutive floats (N = 2, 4, 8) of a position-order row: 8/16-byte vector accesses
template <int N>
__device__ __forceinline__ void ld_row(const float* __restrict__ src, float (&v)[N]) {
  if constexpr (N == 2) {
    const float2 x = *reinterpret_cast<const float2*>(src);
    v[0] = x.x;
    v[1] = x.y;
  } else {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      const float4 x = *reinterpret_cast<const float4*>(src + i);
      v[i] = x.x;
      v[i + 1] = x.y;
      v[i + 2] = x.z;
      v[i + 3] = x.w;
    }
  }
}
template <int N>
__device__ __forceinline__ void st_row(float* __restrict__ dst, const float (&v)[N]) {
  if constexpr (N == 2) {
    *reinterpret_cast<float2*>(dst) = make_float2(v[0], v[1]);
  } else {
#pragma unroll
    for (int i = 0; i < N; i += 4)
      *reinterpret_cast<float4*>(dst + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
  }
}

// The same at byte offset `lo` from a wave-uniform base (ld_lane / st_lane: saddr form)
template <int N>
__device__ __forceinline__ void ld_row(const float* __restrict__ base, uint32_t lo, float (&v)[N]) {
  if constexpr (N == 2) {
    const float2 x = ld_lane(reinterpret_cast<const float2*>(base), lo);
    v[0] = x.x;
    v[1] = x.y;
  } else {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      const float4 x = ld_lane(reinterpret_cast<const float4*>(base), lo + 4 * i);
      v[i] = x.x;
      v[i + 1] = x.y;
      v[i + 2] = x.z;
      v[i + 3] = x.w;
    }
  }
}
template <int N>
__device__ __forceinline__ void st_row(float* __restrict__ base, uint32_t lo, const float (&v)[N]) {
  if constexpr (N == 2) {
    st_lane(reinterpret_cast<float2*>(base), lo, make_float2(v[0], v[1]));
  } else {
#pragma unroll
    for (int i = 0; i < N; i += 4)
      st_lane(reinterpret_cast<float4*>(base), lo + 4 * i,
              make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]));
  }
}

// The same store written through this XCD's L2 (agent-scope sc1 buffer stores): the line is not
// left dirty in L2, so the end-of-launch write-back has less to drain (the S-step's S, mS, vS
// rows are 25 MB per launch at C3; MI355X_MICROARCH.md prices a boundary at +B / 6 TB/s for B
// dirty bytes).  Byte offsets from `base` below 2^31.
#ifndef QSC_WT_S
#define QSC_WT_S 1
#endif
template <int N>
__device__ __forceinline__ void st_row_wt(float* base, uint32_t lo, const float (&v)[N]) {
#if QSC_WT_S
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  typedef unsigned u2v __attribute__((ext_vector_type(2)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff,
                                                                     0x00020000);
  if constexpr (N == 2) {
    const u2v w = {__float_as_uint(v[0]), __float_as_uint(v[1])};
    __builtin_amdgcn_raw_buffer_store_b64(w, r, lo, 0, 16);  // aux 16: sc1
  } else {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      const u4v w = {__float_as_uint(v[i]), __float_as_uint(v[i + 1]), __float_as_uint(v[i + 2]),
                     __float_as_uint(v[i + 3])};
      __builtin_amdgcn_raw_buffer_store_b128(w, r, lo + 16 * (i / 4), 0, 16);
    }
  }
#else
  st_row<N>(base, lo, v);
#endif
}

// Per-slice registers read from HBM: the first group of entry chunks, S[:, q] and (fused Adam)
// the moments of the lane's rows.  Two sets live at once (current + prefetched next slice).
template <int RP, typename E, bool ADAM>
struct SliceIn {
  typename Ent<E>::V2 buf[kGroupS];
  float sv[RP];
  float mv[RP / 2], vv[RP / 2];
  int j1;
  const typename Ent<E>::V2* src;  // the slice's entries (wave-uniform; lanes add SliceLane::ent)

  __device__ __forceinline__ void assign(const SliceIn& o) {
#pragma unroll
    for (int i = 0; i < kGroupS; ++i) buf[i] = o.buf[i];
#pragma unroll
    for (int r = 0; r < RP; ++r) sv[r] = o.sv[r];
    if constexpr (ADAM) {
#pragma unroll
      for (int i = 0; i < RP / 2; ++i) {
        mv[i] = o.mv[i];
        vv[i] = o.vv[i];
      }
    }
    j1 = o.j1;
    src = o.src;
  }
};

// Issue every global read of slice s for this lane (unconditional loads: static vmcnt).
// Entries: the lane's half (entries 2h, 2h+1) of its position's chunk in each chunk row of
// QSC_SLICE positions (2 * QSC_SLICE halves per row), the first kGroupS rows.
// Position-order rows are [Pp][RP]: the lane reads its pixel's whole S row and the half
// [h*RP/2, (h+1)*RP/2) of the Adam moments it will update.
// Per-lane byte offsets of the S-pass accesses (constant for a lane): its entry half within a
// chunk row, its pixel's S row and its half of that row within a slice's block of rows.
struct SliceLane {
  uint32_t ent, row, half;
};
template <int RP, typename E>
__device__ __forceinline__ SliceLane slice_lane(int p, int h) {
  SliceLane l;
  l.ent = (uint32_t)(2 * p + h) * (uint32_t)sizeof(typename Ent<E>::V2);
  l.row = (uint32_t)(p * RP) * 4u;
  l.half = l.row + (uint32_t)(h * (RP / 2)) * 4u;
  return l;
}

template <int RP, typename E, bool ADAM>
__device__ __forceinline__ void slice_load(SliceIn<RP, E, ADAM>& in, const E* __restrict__ ent,
                                           const int* __restrict__ width,
                                           const int64_t* __restrict__ off, int s,
                                           const SliceLane& ln, const float* __restrict__ S,
                                           const float* __restrict__ mS,
                                           const float* __restrict__ vS) {
  using V2 = typename Ent<E>::V2;
  // both slice words read before either is used: one scalar-cache round trip, not two in a
  // chain (the entry reads below depend on both; at the start of a launch this chain is the
  // critical path to the first slice's data)
  const int64_t o = off[s];
  const int wd = width[s];
  in.j1 = wd >> 2;
  in.src = reinterpret_cast<const V2*>(ent + o);
  const int jlast = max(in.j1 - 1, 0);
#pragma unroll
  for (int i = 0; i < kGroupS; ++i)
    in.buf[i] = ld_lane(in.src + (int64_t)min(i, jlast) * (2 * QSC_SLICE), ln.ent);
  const int64_t blk = (int64_t)s * QSC_SLICE * RP;  // the slice's rows (uniform)
  ld_row<RP>(S + blk, ln.row, in.sv);
  if constexpr (ADAM) {
    ld_row<RP / 2>(mS + blk, ln.half, in.mv);
    ld_row<RP / 2>(vS + blk, ln.half, in.vv);
  }
}

// Persistent S-pass: a grid sized to the resident waves; each wave reads slice i+1 while it
// computes slice i, so HBM traffic and arithmetic overlap for the whole pass.  Per-slice NLL /
// ||S_new||^2 partials (DPP wave sums) keep the reductions' order independent of the grid.
template <int RP, typename E, int KIND, bool LOG, bool ADAM>
__global__ void __launch_bounds__(kSBlock, (OccS<RP, (int)sizeof(E), QSC_SPASS_WAVES>::v)) spass_kernel(
    const E* __restrict__ ent, const int* __restrict__ width, const int64_t* __restrict__ off,
    int nslices, Lik lk, Edges E_, int nbins, int R, int K, int Pp, float* __restrict__ S,
    const float* __restrict__ C, float* __restrict__ dS, float* __restrict__ mS,
    float* __restrict__ vS, qsc_adam ad, float lambda_s, qsc_state* __restrict__ st,
    float* __restrict__ part_nll, float* __restrict__ part_nsq, int* __restrict__ sched,
    AdamCache* __restrict__ acache, int ck, int nck) {
  constexpr int CP = TP<RP, KIND>::v;
  constexpr int RH = RP / 2;  // row elements updated per lane (half row)
  // linear models evaluate the entries in a scaled form (lik_grad2)
  const float own_scale = own_scale_of<KIND, LOG>(lk);
  // all LDS carved from the 16-B aligned dynamic region (no statics ahead of it)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Scalars& sc = *reinterpret_cast<Scalars*>(smem);            // 32 B reserved
  float* Cl = smem + 8;                                        // [K][CP] (signed rows: [2K+1])
  float2* El = reinterpret_cast<float2*>(Cl + (size_t)table_floats<RP, KIND>(K));  // [nbins]


  // a wave = one slice of QSC_SLICE (32) pixel positions at a time, two lanes per pixel: lane
  // half h takes entries 2h, 2h+1 of every 4-entry chunk of the pixel's list; the halves'
  // partial dS are summed by a lane swap and each half then updates its half of the pixel's row
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int p = lane & (QSC_SLICE - 1), h = lane >> 5;
  const int W = gridDim.x * kSWaves;
  const int w = blockIdx.x * kSWaves + wave;
  // Static slice schedule: wave w of W takes slices w, 2W-1-w, 2W+w, 4W-1-w, ... (snake order
  // over the count-sorted slices balances the per-wave work)
  auto slice_of = [&](int t) { return t * W + ((t & 1) ? (W - 1 - w) : w); };
  STAMP(w, 0);
  RSTAMP(w, 28);
#if QSC_DIAG_STAMPS
  if (lane == 0 && w < kStampWaves) {
    g_stamps[w * kStamps + 26] = __builtin_amdgcn_s_getreg(0xF804);  // HW_ID: CU / SIMD / wave slot
    g_stamps[w * kStamps + 27] = __builtin_amdgcn_s_getreg(0xF814);  // XCC_ID
  }
#endif
  (void)sched;
  int s = slice_of(0);
  // 1. C^T tile reads first (the LDS staging below waits only for them), then the first slice
  const int k0 = threadIdx.x;
  float c0[RP];
#pragma unroll
  for (int r = 0; r < RP; ++r) c0[r] = C[(int64_t)min(r, R - 1) * K + min(k0, K - 1)];
  const float2 e0 = stages_edges<KIND>() ? E_.e[min(k0, nbins - 1)] : float2{};
  __builtin_amdgcn_sched_barrier(0);
  SliceIn<RP, E, ADAM> cur;
  const SliceLane ln = slice_lane<RP, E>(p, h);
  // unconditional (a wave without slices reads slice 0): a static load count lets the C^T
  // staging below wait for its own reads only
  slice_load(cur, ent, width, off, s < nslices ? s : 0, ln, S, mS, vS);
  // 2. stage C^T (rows padded to CP) and the bin edges in LDS
  {
    // branch-free (threads past K rewrite row K-1 with its own values), so the C^T reads stay
    // ahead of the slice reads
    const int kw = min(k0, K - 1);
#pragma unroll
    for (int r = 0; r < RP; r += 4)
      put_row4<RP, KIND>(Cl, K, kw, r,
                         make_float4(r < R ? c0[r] : 0.0f, r + 1 < R ? c0[r + 1] : 0.0f,
                                     r + 2 < R ? c0[r + 2] : 0.0f, r + 3 < R ? c0[r + 3] : 0.0f),
                         lk.ob_thr);
  }
  for (int k = k0 + kSBlock; k < K; k += kSBlock) {
    float v[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) v[r] = (r < R) ? C[(int64_t)r * K + k] : 0.0f;
#pragma unroll
    for (int r = 0; r < RP; r += 4)
      put_row4<RP, KIND>(Cl, K, k, r, make_float4(v[r], v[r + 1], v[r + 2], v[r + 3]), lk.ob_thr);
  }
  put_pad_row<RP, KIND>(Cl, K);
  if constexpr (stages_edges<KIND>()) {
    El[min(k0, nbins - 1)] = e0;  // branch-free like C^T
    for (int b = k0 + kSBlock; b < nbins; b += kSBlock) El[b] = E_.e[b];
  }
  if (threadIdx.x == 0) {
    if (ADAM) {
      const float nrm = sqrtf(st->normsq_s);
      sc.coef = nrm > 0.0f ? lambda_s / nrm : 0.0f;
      const int step = st->step_s + 1;
      sc.as = adam_scalars_cached(acache[step & 1], ad, step);
    }
    if (blockIdx.x == 0) {
      // book-keeping (fields no block of this kernel reads): see qsc_state
      int pend = st->pending;
      if (pend & QSC_PEND_C) st->step_c += 1;
      pend &= ~QSC_PEND_C;
      st->pending = pend | QSC_PEND_SNLL | (ADAM ? QSC_PEND_SUPD : 0);
      st->normsq_s_prev = st->normsq_s;
      st->iter += 1;
    }
  }
  __syncthreads();
  STAMP(w, 1);

  // one slice: the next slice's reads (into q) in flight during this slice's (c) arithmetic;
  // the loop below alternates the two register sets instead of copying q into c
  int i = 0;
  auto one_slice = [&](SliceIn<RP, E, ADAM>& c, SliceIn<RP, E, ADAM>& q) -> bool {
    const int s1 = slice_of(i + 1);
    const bool more = s1 < nslices;  // wave-uniform
    // 3. next slice's reads (unconditional: a last slice re-reads itself, cache-resident, so
    //    the wait counts stay static)
    QSC_DCHECK(s < nslices && off[s] + (int64_t)width[s] * QSC_SLICE <= lk.dbg_ent[0]);
    slice_load(q, ent, width, off, more ? s1 : s, ln, S, mS, vS);
    STAMP(w, 2 + 3 * i);
    const int64_t blk = (int64_t)s * QSC_SLICE * RP;  // the slice's rows (uniform)
    float sv[RP];  // rows >= R are zero in HBM (position-order padding)
#pragma unroll
    for (int r = 0; r < RP; ++r) sv[r] = c.sv[r];
    f2v own[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) own[j] = f2v{sv[2 * j], sv[2 * j + 1]} * splat2(own_scale);

    // 4. likelihood + gradient over the pixel's observed entries
    f2v accp[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) accp[j] = splat2(0.0f);
    f2v nll = splat2(0.0f);
    walk_halves<RP, E, KIND, LOG>(c.src, ln.ent, 2 * QSC_SLICE, c.j1, c.buf, own, Cl, El, lk,
                                  accp, nll);
    STAMP(w, 3 + 3 * i);
    // the two lane halves' partial dS: v_permlane32_swap (VALU) instead of an LDS shuffle
    float acc[RP];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) {
      acc[2 * j] = accp[j].x;
      acc[2 * j + 1] = accp[j].y;
    }

    // 5. epilogue: fused Adam on the lane's half row, or the raw gradient.  Padding rows
    //    (r >= R) have zero S, C and moments, so Adam keeps them exactly zero.
    float a[RH], pv[RH];
#pragma unroll
    for (int j = 0; j < RH; ++j) {
      a[j] = half_sum_pick(acc[j], acc[RH + j]);
      pv[j] = swap_lo(sv[j], sv[RH + j]);
    }
    if constexpr (ADAM) {
      float m[RH], v[RH];
#pragma unroll
      for (int j = 0; j < RH; ++j) {
        m[j] = c.mv[j];
        v[j] = c.vv[j];
      }
      float nsq = adam_row_fast<RH>(pv, m, v, a, sc.coef, sc.as, ad.project_nonneg != 0);
      st_row_wt<RH>(S + blk, ln.half, pv);
      st_row_wt<RH>(mS + blk, ln.half, m);
      st_row_wt<RH>(vS + blk, ln.half, v);
      nsq = wave_sum_dpp(nsq);
      if (lane == 0) part_nsq[s] = nsq;
    } else {
      // (K-slab, ck > 0: the reduce-scatter layout, one extra slice after every ck slices)
      const int64_t dblk = ck > 0 ? (int64_t)(s + s / ck) * QSC_SLICE * RP : blk;
      st_row_wt<RH>(dS + dblk, ln.half, a);
    }
    const float nll_w = wave_sum_dpp(nll.x + nll.y) * kLn2;
    if (lane == 0) part_nll[s] = nll_w;
    STAMP(w, 4 + 3 * i);
    s = s1;
    ++i;
    return more;
  };
  if (s < nslices) {
    SliceIn<RP, E, ADAM> nxt;
    for (;;) {
      if (!one_slice(cur, nxt)) break;
      if (!one_slice(nxt, cur)) break;
    }
  }
  // the next S-step's scalars (cfinish settles step_s + 1 in between)
  if (ADAM && blockIdx.x == 0 && threadIdx.x == 0) adam_cache_store(acache, ad, st->step_s + 2);
  if constexpr (!ADAM) {
    // K-slab (ck > 0): ||C_slab||^2 of the C this pass read -- the C the next C-step
    // differentiates -- into the extra slice of every rank's chunk of the reduce-scatter buffer,
    // so the reduce-scatter of dS delivers every rank the GLOBAL ||C||^2 with its gradient rows
    // (no all-reduce of its own).  Order of cnorm_sq (thread t < 256 accumulates t, t + 256, ...
    // then the block sum): the same bits as the C-pass's ||C||^2.  (Sc's scratch is free here.)
    if (ck > 0 && blockIdx.x == 0) {
      float s2 = 0.0f;
      if (threadIdx.x < 256)
        for (int i2 = threadIdx.x; i2 < R * K; i2 += 256) {
          const int r = i2 / K, k = i2 - r * K;
          const float c = Cl[k * CP + r];
          s2 = __builtin_fmaf(c, c, s2);
        }
      const float nsq = block_sum(s2, smem);
      if (threadIdx.x == 0)
        for (int c = 0; c < nck; ++c) dS[(int64_t)(c * (ck + 1) + ck) * QSC_SLICE * RP] = nsq;
    }
  }
  STAMP(w, kStampLast);
  RSTAMP(w, 29);
}

// ---------------------------------------------------------------------------------------
// C-pass
// ---------------------------------------------------------------------------------------
// One workgroup per (pixel tile, 64-bin frequency slice): kCParts waves, each walking a part of
// the slice's per-bin entry lists (lane = bin k) against the tile's S rows staged in LDS.
// Small workgroups (several resident per CU, dispatched as others retire) let the hardware
// balance the uneven lists and overlap one group's staging with another's arithmetic.  The
// four quarters are summed in LDS in a fixed order and written as the tile's dC slab rows.
// Block -> (tile, slice) map: the nks slices of a tile are given blocks that the round-robin
// dispatcher places on one XCD (b, b+8, b+16, ...), so the tile's S rows are read from that
// XCD's L2 after the first (speed only; any bijection is correct).
constexpr int kCParts = kCBlock / 64;

template <int RP, typename E, int KIND, bool LOG>
__global__ void __launch_bounds__(kCBlock, (Occ<RP, QSC_CPASS_WAVES>::v)) cpass_kernel(
    const E* __restrict__ ent, const int* __restrict__ width, const int64_t* __restrict__ off,
    const int* __restrict__ kmap, int nks, int PT, int xcd_map, Lik lk, Edges E_, int nbins,
    int R, int K,
    const float* __restrict__ S, const float* __restrict__ C, float* __restrict__ slab,
    float* __restrict__ part_nll, float* __restrict__ cnsq) {
  using T = Ent<E>;
  using V4 = typename T::V4;
  constexpr int SP = TP<RP, KIND>::v;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int TR = table_rows<KIND>(PT);
  float* Sl = smem;                                              // [PT][SP] (signed: [2PT+1])
  float2* El = reinterpret_cast<float2*>(Sl + (size_t)table_floats<RP, KIND>(PT));  // [nbins]
  float* Pl = Sl + (size_t)table_floats<RP, KIND>(PT) + 2 * 256;  // [kCParts][R][64]
  (void)TR;

  float* Nl = Pl + (size_t)kCParts * R * 64;                      // [kCParts]
  int t, ks;
  if (xcd_map) {
    const int j = blockIdx.x >> 3, x = blockIdx.x & 7;
    t = (j / nks) * 8 + x;
    ks = j - (j / nks) * nks;
  } else {
    t = blockIdx.x / nks;
    ks = blockIdx.x - t * nks;
  }
  const int Kp = nks * 64;
  const int part = threadIdx.x >> 6, lane = threadIdx.x & 63;
  [[maybe_unused]] const int wg = blockIdx.x * kCParts + part;  // (diagnostic stamps)
  STAMP(wg, 0);
  RSTAMP(wg, 28);

  // 1. entry read-ahead of this wave's part of the lists and C[:, k], before the staging
  const int64_t wi = (int64_t)t * nks + ks;
  const int W4 = width[wi] >> 2;
  const PartRange pr = part_range(W4, part, kCParts);
  const int j0 = pr.j0, j1 = pr.j1;
  const V4* src = reinterpret_cast<const V4*>(ent + off[wi]);
  const uint32_t lo = (uint32_t)lane * (uint32_t)sizeof(V4);
  V4 buf[kGroup];
  load_group(src, lo, 64, j0, pr.js, max(j1 - 1, 0), buf);
  const int k = kmap[wi * 64 + lane];  // this lane's bin (count-sorted order, include/qsc.h)
  float cv[RP];
#pragma unroll
  for (int r = 0; r < RP; ++r) cv[r] = C[(int64_t)min(r, R - 1) * K + min(k, K - 1)];

  // 2. stage the pixel tile: its rows are whole position slices (qsc_tile_pos, snake-dealt),
  //    each a contiguous run of QSC_SLICE rows in [Pp][RP]; 16-B reads and 16-B LDS writes at
  //    the padded pitch SP
  {
    const float4* __restrict__ src4 = reinterpret_cast<const float4*>(S);
    constexpr int V = RP / 4;  // float4 per row
    const int nt = gridDim.x / nks;
#pragma unroll 4
    for (int i = threadIdx.x; i < PT * V; i += kCBlock) {
      const int ql = i / V, c = i - ql * V;
      put_row4<RP, KIND>(Sl, PT, ql, 4 * c, src4[tile_pos(t, ql, nt) * V + c], lk.ob_thr);
    }
    put_pad_row<RP, KIND>(Sl, PT);
  }
  for (int i = threadIdx.x; i < nbins; i += kCBlock) El[i] = E_.e[i];
  __syncthreads();
  STAMP(wg, 1);

  // 3. likelihood + gradient over the part lists
  const float own_scale = own_scale_of<KIND, LOG>(lk);  // scaled form (lik_grad2)
  f2v own[RP / 2];
#pragma unroll
  for (int j = 0; j < RP / 2; ++j)
    own[j] = f2v{(2 * j < R && k < K) ? cv[2 * j] : 0.0f,
                 (2 * j + 1 < R && k < K) ? cv[2 * j + 1] : 0.0f} * splat2(own_scale);
  f2v accp[RP / 2];
#pragma unroll
  for (int j = 0; j < RP / 2; ++j) accp[j] = splat2(0.0f);
  f2v nll = splat2(0.0f);
#if QSC_CPASS_MASKED
  walk_masked<RP, E, KIND, LOG>(src, lo, 64, j0, j0, j1, pr.js, buf, own, Sl, El, lk, accp, nll);
#else
  walk_groups<RP, E, KIND, LOG>(src, lo, 64, j0, j1, pr.js, buf, own, Sl, El, lk, accp, nll);
#endif
  STAMP(wg, 2);
  const float nll_w = wave_sum_dpp(nll.x + nll.y) * kLn2;
#pragma unroll
  for (int j = 0; j < RP / 2; ++j) {
    if (2 * j < R) Pl[((size_t)part * R + 2 * j) * 64 + lane] = accp[j].x;
    if (2 * j + 1 < R) Pl[((size_t)part * R + 2 * j + 1) * 64 + lane] = accp[j].y;
  }
  if (lane == 0) Nl[part] = nll_w;
  __syncthreads();
  STAMP(wg, 3);

  // 4. fixed-order sum of the parts -> slab rows of this tile / slice
  for (int i = threadIdx.x; i < R * 64; i += kCBlock) {
    float a = Pl[i];
#pragma unroll
    for (int pp = 1; pp < kCParts; ++pp) a += Pl[(size_t)pp * R * 64 + i];
    const int r = i >> 6, l = i & 63;
    slab[((int64_t)t * R + r) * Kp + kmap[wi * 64 + l]] = a;
  }
  if (threadIdx.x == 0) {
    float a = Nl[0];
#pragma unroll
    for (int pp = 1; pp < kCParts; ++pp) a += Nl[pp];
    part_nll[wi] = a;
  }
  if (blockIdx.x == 0) {
    // ||C||^2 for the C update's regulariser (fixed order; C is read-only in this kernel)
    const float nsq = cnorm_sq(C, R * K, Nl);  // Nl's slots are free again
    if (threadIdx.x == 0) *cnsq = nsq;
  }
  STAMP(wg, kStampLast);
  RSTAMP(wg, 29);
}

// ---------------------------------------------------------------------------------------
// C-pass, tile form: one workgroup per pixel tile covering ALL of its k-slices, so the tile's
// S rows are staged in LDS once (not once per 64-bin slice) and the whole grid is resident in
// one round (tiles hold equal mixes of dense and sparse positions, qsc_tile_pos, so the
// workgroups carry equal work).  The NW = blockDim/64 waves take units (k-slice ks, part of
// NP) u = w, w + NW, ...: lane = bin k walks part `part` of the bin's list.  With NP = 1 a
// unit's dC goes straight from registers to the slab; otherwise the NP parts are summed in
// LDS in a fixed order (bitwise deterministic; no atomics).
// ---------------------------------------------------------------------------------------
constexpr int kCTBlock = 1024;
// waves of a rank-16 tile workgroup: 8 (2 per SIMD, 256 VGPRs).  At 16 waves (128 VGPRs) the
// rank-16 walk's 16-float C column, accumulators and pipelined gather rows spill 14-62 VGPRs
// (tools/isa_stats.py), which made the c4k C-pass 2.3x slower per entry than rank 8
#ifndef QSC_CTILE_W16
#define QSC_CTILE_W16 8
#endif
#ifndef QSC_CTILE_SREG
#define QSC_CTILE_SREG 4
#endif
#ifndef QSC_CTILE_CT
#define QSC_CTILE_CT 1
#endif
template <int RP>
struct CTBlock {
  static constexpr int w = RP > 8 ? QSC_CTILE_W16 : kCTBlock / 64;  // max waves
  static constexpr int v = 64 * w;
};

template <int RP, typename E, int KIND, bool LOG>
__global__ void __launch_bounds__(CTBlock<RP>::v) cpass_tile_kernel(
    const E* __restrict__ ent, const int* __restrict__ width, const int64_t* __restrict__ off,
    const int* __restrict__ kmap, int nks, int NP, int PT, Lik lk, Edges E_, int nbins, int R,
    int K, int ct_in,
    const float* __restrict__ S, const float* __restrict__ C, float* __restrict__ slab,
    float* __restrict__ part_nll, float* __restrict__ cnsq, float* __restrict__ snsq_out) {
  using T = Ent<E>;
  using V4 = typename T::V4;
  constexpr int SP = TP<RP, KIND>::v;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int NW = blockDim.x >> 6;
  const int U = nks * NP;
  const int TR = table_rows<KIND>(PT);
  float* Sl = smem;                                              // [PT][SP] (signed: [2PT+1])
  float2* El = reinterpret_cast<float2*>(Sl + (size_t)table_floats<RP, KIND>(PT));  // [nbins]
  float* Pl = Sl + (size_t)table_floats<RP, KIND>(PT) + 2 * 256;  // [U][R][64]   (NP > 1)
  (void)TR;

  float* Nl = Pl + (NP > 1 ? (size_t)U * R * 64 : 0);             // [U] / [NW]
  // (ct) C^T staged next to the tile, [K][RP] (rows r >= R unread), for the units' C columns
  // (not for 32-bit entries below rank 16: their 16-wave walk has no VGPRs to spare)
  float* Ctl = Nl + ((max(U, 16) + 3) & ~3);
  const bool ct = (RP > 8 || sizeof(E) == 2) && ct_in != 0;
  const int t = blockIdx.x;
  const int Kp = nks * 64;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const float own_scale = own_scale_of<KIND, LOG>(lk);  // scaled form (lik_grad2)
  [[maybe_unused]] const int wg = blockIdx.x * CTBlock<RP>::w + w;  // (diagnostic stamps)
  STAMP(wg, 0);
  RSTAMP(wg, 28);

  // 1. read-ahead of the first unit's entries and C column, ahead of the staging
  int u = w;
  V4 buf[kGroup];
  float cv[RP];
  int wi = 0, j0 = 0, j1 = 0, js = 1, k = 0;
  const V4* src = nullptr;
  const uint32_t lo = (uint32_t)lane * (uint32_t)sizeof(V4);
  // the unit's C column: from the staged C^T (ct; after the staging barrier) or from C
  auto unit_cols = [&]() {
    if (ct) {
#pragma unroll
      for (int r = 0; r < RP; r += 4) {
        const float4 q = *reinterpret_cast<const float4*>(Ctl + (size_t)min(k, K - 1) * RP + r);
        cv[r] = q.x;
        cv[r + 1] = q.y;
        cv[r + 2] = q.z;
        cv[r + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int r = 0; r < RP; ++r) cv[r] = C[(int64_t)min(r, R - 1) * K + min(k, K - 1)];
    }
  };
  auto unit_begin = [&](int uu, bool cols) {
    const int ks = uu / NP, part = uu - ks * NP;
    wi = t * nks + ks;
    const int W4 = width[wi] >> 2;
    const PartRange pr = part_range(W4, part, NP);
    j0 = pr.j0;
    j1 = pr.j1;
    js = pr.js;
    src = reinterpret_cast<const V4*>(ent + off[wi]);
    QSC_DCHECK(off[wi] + (int64_t)width[wi] * 64 <= lk.dbg_ent[1]);
    load_group(src, lo, 64, j0, js, max(j1 - 1, 0), buf);
    k = kmap[wi * 64 + lane];  // this lane's bin (count-sorted order)
    QSC_DCHECK(k >= 0 && k < Kp);
    if (cols) unit_cols();
  };
  // the tile's S rows are read first, into registers when they fit QSC_CTILE_SREG float4 per
  // thread: the unit's reads below wait on their own dependent reads (bounds -> entries, bin ->
  // C column), so rows issued after them arrived one round trip later
  const float4* __restrict__ src4 = reinterpret_cast<const float4*>(S);
  constexpr int V = RP / 4;  // float4 per row
  // (not for 32-bit entries below rank 16: their 16-wave walk has no VGPRs to spare)
  constexpr bool kSRok = QSC_CTILE_SREG > 0 && (RP > 8 || sizeof(E) == 2);
  constexpr int kSR = kSRok ? QSC_CTILE_SREG : 1;
  const bool sreg = kSRok && PT * V <= kSR * (int)blockDim.x;
  float4 srow[kSR];
  if (sreg) {
#pragma unroll
    for (int q = 0; q < kSR; ++q) {
      const int i = (int)threadIdx.x + q * (int)blockDim.x;
      const int ql = i / V, c = i - ql * V;
      if (i < PT * V) srow[q] = src4[tile_pos(t, ql, (int)gridDim.x) * V + c];
    }
  }
  // (ct) the C^T reads: no dependency, so they ride with the S rows' round trip
  constexpr int kCT = 4;  // C floats per thread held in registers (R K <= kCT * blockDim)
  float ctv[kCT];
  if (ct) {
#pragma unroll
    for (int q = 0; q < kCT; ++q) {
      const int i = (int)threadIdx.x + q * (int)blockDim.x;
      if (i < R * K) ctv[q] = C[i];
    }
  }
  if (u < U) unit_begin(u, !ct);

  // 2. stage the pixel tile (whole position slices, 16-B reads / writes at pitch SP)
  {
    const int nt = gridDim.x;
    if (ct) {
#pragma unroll
      for (int q = 0; q < kCT; ++q) {
        const int i = (int)threadIdx.x + q * (int)blockDim.x;
        if (i < R * K) {
          const int r = i / K, kk = i - r * K;
          Ctl[(size_t)kk * RP + r] = ctv[q];
        }
      }
    }
    if (sreg) {
#pragma unroll
      for (int q = 0; q < kSR; ++q) {
        const int i = (int)threadIdx.x + q * (int)blockDim.x;
        const int ql = i / V, c = i - ql * V;
        if (i < PT * V) put_row4<RP, KIND>(Sl, PT, ql, 4 * c, srow[q], lk.ob_thr);
      }
    } else {
#pragma unroll 4
      for (int i = threadIdx.x; i < PT * V; i += blockDim.x) {
        const int ql = i / V, c = i - ql * V;
        put_row4<RP, KIND>(Sl, PT, ql, 4 * c, src4[tile_pos(t, ql, nt) * V + c], lk.ob_thr);
      }
    }
    put_pad_row<RP, KIND>(Sl, PT);
  }
  for (int i = threadIdx.x; i < nbins; i += blockDim.x) El[i] = E_.e[i];
  __syncthreads();
  STAMP(wg, 1);
  if (ct && u < U) unit_cols();

  // 3. units: likelihood + gradient over the part lists
  for (; u < U; u += NW) {
    f2v own[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j)
      own[j] = f2v{(2 * j < R && k < K) ? cv[2 * j] : 0.0f,
                   (2 * j + 1 < R && k < K) ? cv[2 * j + 1] : 0.0f} * splat2(own_scale);
    f2v accp[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) accp[j] = splat2(0.0f);
    f2v nll = splat2(0.0f);
    walk_groups<RP, E, KIND, LOG>(src, lo, 64, j0, j1, js, buf, own, Sl, El, lk, accp, nll);
    const float nll_w = wave_sum_dpp(nll.x + nll.y) * kLn2;
    if (NP == 1) {
      // the unit is the whole (tile, k-slice): its slab rows straight from registers
#pragma unroll
      for (int j = 0; j < RP / 2; ++j) {
        if (2 * j < R) slab[((int64_t)t * R + 2 * j) * Kp + k] = accp[j].x;
        if (2 * j + 1 < R) slab[((int64_t)t * R + 2 * j + 1) * Kp + k] = accp[j].y;
      }
      if (lane == 0) part_nll[wi] = nll_w;
    } else {
#pragma unroll
      for (int j = 0; j < RP / 2; ++j) {
        if (2 * j < R) Pl[((size_t)u * R + 2 * j) * 64 + lane] = accp[j].x;
        if (2 * j + 1 < R) Pl[((size_t)u * R + 2 * j + 1) * 64 + lane] = accp[j].y;
      }
      if (lane == 0) Nl[u] = nll_w;
    }
    if (u + NW < U) unit_begin(u + NW, true);
  }
  STAMP(wg, 2);

  // 3b. (qsc_cpass_nsq, K-slab) every slice's ||S||^2 partial from the staged tile, in
  //     slice_nsq_kernel's lane mapping (lane p + 32 h: position p, half row h) and order, so
  //     the values are bit-identical to qsc_slice_nsq's / the shard updates' partials
  if (snsq_out) {
    constexpr int RH = RP / 2;
    const int nsl = PT / QSC_SLICE, nt = gridDim.x;
    const int p = lane & (QSC_SLICE - 1), h = lane >> 5;
    for (int ls = w; ls < nsl; ls += NW) {
      const float* row = Sl + (size_t)(ls * QSC_SLICE + p) * SP + h * RH;
      float nsq = 0.0f;
#pragma unroll
      for (int j = 0; j < RH; ++j) nsq = __builtin_fmaf(row[j], row[j], nsq);
      nsq = wave_sum(nsq);
      if (lane == 0) snsq_out[tile_pos(t, ls * QSC_SLICE, nt) / QSC_SLICE] = nsq;
    }
  }

  // 4. fixed-order sum of the parts -> slab rows of this tile (NP > 1)
  if (NP > 1) {
    __syncthreads();
    STAMP(wg, 3);
    for (int i = threadIdx.x; i < nks * R * 64; i += blockDim.x) {
      const int ks = i / (R * 64), rl = i - ks * (R * 64);
      const float* p = Pl + (size_t)ks * NP * R * 64 + rl;
      float a = p[0];
      for (int pp = 1; pp < NP; ++pp) a += p[(size_t)pp * R * 64];
      const int r = rl >> 6, l = rl & 63;
      slab[((int64_t)t * R + r) * Kp + kmap[((int64_t)t * nks + ks) * 64 + l]] = a;
    }
    for (int ks = threadIdx.x; ks < nks; ks += blockDim.x) {
      float a = Nl[ks * NP];
      for (int pp = 1; pp < NP; ++pp) a += Nl[ks * NP + pp];
      part_nll[t * nks + ks] = a;
    }
  }
  if (blockIdx.x == 0) {
    // ||C||^2 for the C update's regulariser (fixed order; C is read-only in this kernel)
    __syncthreads();
    const float nsq = cnorm_sq(C, R * K, Nl);  // Nl's slots are free again
    if (threadIdx.x == 0) *cnsq = nsq;
  }
  STAMP(wg, kStampLast);
  RSTAMP(wg, 29);
}

// LDS bytes of cpass_tile_kernel
// pitch (floats) and row count of a gather table (sr: signed rows)
inline int tpitch(int R, bool sr) {
  const int RP = R <= 4 ? 4 : (R <= 8 ? 8 : 16);
  return (sr || RP > 4) ? RP + 4 : 4;
}
inline size_t trows(int rows, bool sr) { return sr ? (size_t)sr_rows(rows) : (size_t)rows; }
// floats of a gather table
inline size_t tfloats(int rows, int R, bool sr) { return trows(rows, sr) * tpitch(R, sr); }

size_t cpass_tile_lds(int PT, int R, int nks, int NP, bool sr) {
  const size_t U = (size_t)nks * NP;
  return tfloats(PT, R, sr) * 4 + 2 * 256 * 4 + (NP > 1 ? U * R * 64 * 4 : 0) +
         std::max<size_t>(U, 16) * 4;
}

#ifndef QSC_CPASS_TILE
#define QSC_CPASS_TILE 1
#endif
#ifndef QSC_CTILE_MAXW
#define QSC_CTILE_MAXW 16
#endif

// ---------------------------------------------------------------------------------------
// Fused S-step + next C-pass, one workgroup per C-pass pixel tile (16 waves; 8 at rank 16).
// The tile's whole position slices (tile_pos) get their S-step first -- likelihood, dS and
// Adam exactly as spass_kernel, wave w taking the tile's slices w, 2*16-1-w, ... (snake over
// the count-sorted slices) -- and the new S rows are written to HBM (S, mS, vS) AND into the
// LDS tile; after one barrier the same workgroup runs the tile's C-pass units exactly as
// cpass_tile_kernel, at the new S, for the NEXT iteration's C-step.  So one launch replaces
// spass + cpass: no kernel boundary between them and no re-read / staging of the S tile (the
// C-pass of iteration i+1 reads only S_i of its own tile, and C_i, which the S-step also used).
// Kernel sequence semantics are unchanged: spass_i then cpass_{i+1} (same partials, same
// state protocol), so a solver runs cpass+cfinish, then (fused + cfinish) x (n-1), then spass.
// ---------------------------------------------------------------------------------------
// fused launch block: 16 waves (4 per SIMD, 128 VGPRs) up to rank 8; 8 waves at rank 16, whose
// two slice register sets and 16-float rows need up to 256 VGPRs (2 waves per SIMD)

template <int RP>
struct FusedBlock {
  static constexpr int v = RP > 8 ? 512 : 64 * QSC_FUSED_WAVES;
  static constexpr int wpe = RP > 8 ? 2 : (QSC_FUSED_WAVES + 3) / 4;  // waves per SIMD
};

// (device-function form: the 2 KB edge table by reference; kernel form below: by value --
// a kernel argument is never a reference, which would hand the device a host address)
#define QSC_SCF_PARAMS                                                                         \
  const E *__restrict__ s_ent, const int *__restrict__ s_width, const int64_t *__restrict__ s_off, \
      const E *__restrict__ c_ent, const int *__restrict__ c_width,                                \
      const int64_t *__restrict__ c_off, const int *__restrict__ c_kmap, int nks, int NP, int PT,  \
      Lik lk, const Edges &E_, int nbins, int R, int K, float *__restrict__ S,                    \
      const float *__restrict__ C,                                                                \
      float *__restrict__ mS, float *__restrict__ vS, qsc_adam ad, float lambda_s,                \
      qsc_state *__restrict__ st, float *__restrict__ part_nll_s, float *__restrict__ part_nsq_s, \
      float *__restrict__ slab, float *__restrict__ part_nll_c, float *__restrict__ cnsq,         \
      AdamCache *__restrict__ acache
#define QSC_SCF_KPARAMS                                                                        \
  const E *__restrict__ s_ent, const int *__restrict__ s_width, const int64_t *__restrict__ s_off, \
      const E *__restrict__ c_ent, const int *__restrict__ c_width,                                \
      const int64_t *__restrict__ c_off, const int *__restrict__ c_kmap, int nks, int NP, int PT,  \
      Lik lk, Edges E_, int nbins, int R, int K, float *__restrict__ S,                           \
      const float *__restrict__ C,                                                                \
      float *__restrict__ mS, float *__restrict__ vS, qsc_adam ad, float lambda_s,                \
      qsc_state *__restrict__ st, float *__restrict__ part_nll_s, float *__restrict__ part_nsq_s, \
      float *__restrict__ slab, float *__restrict__ part_nll_c, float *__restrict__ cnsq,         \
      AdamCache *__restrict__ acache
#define QSC_SCF_ARGS                                                                            \
  s_ent, s_width, s_off, c_ent, c_width, c_off, c_kmap, nks, NP, PT, lk, E_, nbins, R, K, S, C, mS, \
      vS, ad, lambda_s, st, part_nll_s, part_nsq_s, slab, part_nll_c, cnsq, acache


// One pixel tile t of nt of the fused launch (scfused_kernel: t = the workgroup).  C is
// read-only here.
template <int RP, typename E, int KIND, bool LOG>
__device__ __forceinline__ void scfused_tile(QSC_SCF_PARAMS, const int t, const int nt,
                                             const unsigned tidx) {
  using V4 = typename Ent<E>::V4;
  constexpr int CP = TP<RP, KIND>::v;  // C^T row pitch == S tile row pitch
  constexpr int RH = RP / 2;
  constexpr bool ADAM = true;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Scalars& sc = *reinterpret_cast<Scalars*>(smem);                // 32 B
  float* Cl = smem + 8;                                            // [K][CP] (signed: 2K+1)
  float2* El = reinterpret_cast<float2*>(Cl + (size_t)table_floats<RP, KIND>(K));  // [256]
  float* Sl = reinterpret_cast<float*>(El + 256);                   // [PT][CP] (signed: 2PT+1)
  float* Pl = Sl + (size_t)table_floats<RP, KIND>(PT);              // [U][R][64]  (NP > 1)

  const int NW = blockDim.x >> 6;
  const int U = nks * NP;
  float* Nl = Pl + (NP > 1 ? (size_t)U * R * 64 : 0);               // [max(U,16)]
  const int Kp = nks * 64;
  const int w = __builtin_amdgcn_readfirstlane(tidx >> 6), lane = tidx & 63;
  const int p = lane & (QSC_SLICE - 1), h = lane >> 5;
  const float own_scale = own_scale_of<KIND, LOG>(lk);
  const int nsl = PT / QSC_SLICE;  // slices per tile
  // this wave's n-th slice of the tile (local index) and its global slice
  auto local_of = [&](int n) { return n * NW + ((n & 1) ? (NW - 1 - w) : w); };
  auto global_of = [&](int i) { return i * nt + ((i & 1) ? (nt - 1 - t) : t); };
  [[maybe_unused]] const int wg = t * (FusedBlock<RP>::v / 64) + w;  // (stamps)
  STAMP(wg, 0);
  RSTAMP(wg, 28);
#if QSC_DIAG_STAMPS
  if (lane == 0 && wg < kStampWaves) g_stamps[wg * kStamps + 26] = __builtin_amdgcn_s_getreg(0xF804);
#endif

  // 1. C^T / edge / state reads first (the LDS staging then waits only for them: vmcnt
  //    retires in issue order), then the first slice's reads, then the staging
  const int k0 = tidx;
#if QSC_CT_VEC
  // C^T from 16-B reads of the [R][K] C: thread i holds C's flat floats 4i..4i+3 (one row r,
  // four consecutive bins) and writes them transposed; 32x fewer read instructions than a
  // float per (thread, row)
  const int n4 = (R * K) >> 2;
  const bool cvec = (K & 3) == 0 && ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
  float4 cq = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float c0[RP];
  if (cvec) {
    cq = reinterpret_cast<const float4*>(C)[min(k0, n4 - 1)];
  } else {
#pragma unroll
    for (int r = 0; r < RP; ++r) c0[r] = C[(int64_t)min(r, R - 1) * K + min(k0, K - 1)];
  }
#else
  float c0[RP];
#pragma unroll
  for (int r = 0; r < RP; ++r) c0[r] = C[(int64_t)min(r, R - 1) * K + min(k0, K - 1)];
#endif
  const float2 e0 = stages_edges<KIND>() ? E_.e[min(k0, nbins - 1)] : float2{};
#if QSC_KMAP_PF
  // the bins of this thread's first two part-sum outputs (step 4), read now: at the tail they
  // would be a dependent global read after the last unit
  const int nps = nks * R * 64;
  int km_pf[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = min(k0 + j * (int)blockDim.x, nps - 1);
    const int ks = i / (R * 64), l = (i - ks * (R * 64)) & 63;
    km_pf[j] = c_kmap[((int64_t)t * nks + ks) * 64 + l];
  }
#endif
  float nsq_s = 0.0f;
  int step_s = 0;
  AdamCache ac0{}, ac1{};
  if (tidx == 0) {
    nsq_s = st->normsq_s;
    step_s = st->step_s;
    ac0 = acache[0];  // both slots: no dependent read on step_s
    ac1 = acache[1];
  }
  __builtin_amdgcn_sched_barrier(0);
  STAMP(wg, 13);  // (the C^T, edge, state reads are issued)
  int il = local_of(0);
  SliceIn<RP, E, ADAM> cur;
  const SliceLane ln = slice_lane<RP, E>(p, h);
  // First reads before the staging: waves w < QSC_EARLY_WAVES read their first slice now, the
  // others after the staging barrier.  The C^T reads the staging waits for take 2.5-3 us at a
  // launch's start (profiles/r05/stamps_f.log), long enough to cover every wave's first slice:
  // with all 16 waves early the fused launch is 0.6-0.9 us shorter at C3 than with the oldest
  // wave of each SIMD only (QSC_EARLY_WAVES=4, round 3's choice when the staging was shorter;
  // profiles/r05/ab_early_waves.log).
  const bool early = w < QSC_EARLY_WAVES;
  auto stage = [&]() {
    STAMP(wg, 14);  // (the wave's first-slice reads, if early, are issued)
#if QSC_CT_VEC
    if (cvec) {
      const int Ko = sr_off(K);  // the negated half of a signed-row C^T table
      auto put = [&](int i, const float4& v) {
        const int f = 4 * i, r = f / K, k = f - r * K;
        Cl[k * CP + r] = v.x;
        Cl[(k + 1) * CP + r] = v.y;
        Cl[(k + 2) * CP + r] = v.z;
        Cl[(k + 3) * CP + r] = v.w;
        if constexpr (is_sr(KIND)) {
          Cl[(Ko + k) * CP + r] = -v.x;
          Cl[(Ko + k + 1) * CP + r] = -v.y;
          Cl[(Ko + k + 2) * CP + r] = -v.z;
          Cl[(Ko + k + 3) * CP + r] = -v.w;
        }
      };
      if (k0 < n4) put(k0, cq);
      for (int i = k0 + (int)blockDim.x; i < n4; i += blockDim.x)
        put(i, reinterpret_cast<const float4*>(C)[i]);
      for (int i = k0; i < K * (RP - R); i += blockDim.x) {  // rows R..RP-1 are zero
        const int k = i / (RP - R), r = R + (i - k * (RP - R));
        Cl[k * CP + r] = 0.0f;
        if constexpr (is_sr(KIND)) Cl[(Ko + k) * CP + r] = -0.0f;
      }
      if constexpr (is_sr(KIND))
        for (int k = k0; k < K; k += blockDim.x) put_th<RP, KIND>(Cl, K, k, lk.ob_thr);
    } else
#endif
    {
      const int kw = min(k0, K - 1);  // branch-free: threads past K rewrite row K-1
#pragma unroll
      for (int r = 0; r < RP; r += 4)
        put_row4<RP, KIND>(Cl, K, kw, r,
                           make_float4(r < R ? c0[r] : 0.0f, r + 1 < R ? c0[r + 1] : 0.0f,
                                       r + 2 < R ? c0[r + 2] : 0.0f, r + 3 < R ? c0[r + 3] : 0.0f),
                           lk.ob_thr);
      for (int k = k0 + (int)blockDim.x; k < K; k += blockDim.x) {
        float v[RP];
#pragma unroll
        for (int r = 0; r < RP; ++r) v[r] = (r < R) ? C[(int64_t)r * K + k] : 0.0f;
#pragma unroll
        for (int r = 0; r < RP; r += 4)
          put_row4<RP, KIND>(Cl, K, k, r, make_float4(v[r], v[r + 1], v[r + 2], v[r + 3]),
                             lk.ob_thr);
      }
    }
    put_pad_row<RP, KIND>(Cl, K);
    if constexpr (is_sr(KIND)) {
      // the S tile's threshold column and pad row (its S values are written by the S-step)
      for (int q = k0; q < PT; q += blockDim.x) put_th<RP, KIND>(Sl, PT, q, lk.ob_thr);
      put_pad_row<RP, KIND>(Sl, PT);
    }
    if constexpr (stages_edges<KIND>()) {
      El[min(k0, nbins - 1)] = e0;
      for (int b = k0 + (int)blockDim.x; b < nbins; b += blockDim.x) El[b] = E_.e[b];
    }
    STAMP(wg, 10);  // C^T rows written (its reads landed)
    if (tidx == 0) {
      const float nrm = sqrtf(nsq_s);
      sc.coef = nrm > 0.0f ? lambda_s / nrm : 0.0f;
      sc.as = adam_scalars_cached(((step_s + 1) & 1) ? ac1 : ac0, ad, step_s + 1);
      if (t == 0) {
        // book-keeping of spass_kernel (mode 1)
        int pend = st->pending;
        if (pend & QSC_PEND_C) st->step_c += 1;
        pend &= ~QSC_PEND_C;
        st->pending = pend | QSC_PEND_SNLL | QSC_PEND_SUPD;
        st->normsq_s_prev = nsq_s;
        st->iter = st->iter + 1;
      }
    }
    STAMP(wg, 11);  // (wave 0: the scalars are set)
  };
  // (late waves' first reads right after their own staging instead of after the barrier:
  // within noise, round 5, gpurun_out/r05q; not kept)
  if (early) {
    slice_load(cur, s_ent, s_width, s_off, global_of(il < nsl ? il : 0), ln, S, mS, vS);
    stage();
  } else {
    stage();
  }
  __syncthreads();
  if (!early) slice_load(cur, s_ent, s_width, s_off, global_of(il < nsl ? il : 0), ln, S, mS, vS);
  STAMP(wg, 1);
  if (t == 0) {
    // ||C_i||^2 for the next C update's regulariser, from the staged C^T at the start (as a
    // chain of dependent global reads at the end it delayed the last workgroup); the order of
    // cnorm_sq: thread t < 256 accumulates flat indices t, t + 256, ..., then block_sum
    float s2 = 0.0f;
    if (tidx < 256)
      for (int i = tidx; i < R * K; i += 256) {
        const int r = i / K, k = i - r * K;
        const float c = Cl[k * CP + r];
        s2 = __builtin_fmaf(c, c, s2);
      }
    const float nsq = block_sum(s2, Nl);
    if (tidx == 0) *cnsq = nsq;
  }

  // 2. S-step over the wave's slices (next slice's reads in flight; the two register sets
  //    alternate, as in spass_kernel)
  int n = 0;
  auto one_slice = [&](SliceIn<RP, E, ADAM>& c, SliceIn<RP, E, ADAM>& q) -> bool {
    const int il1 = local_of(n + 1);
    const bool more = il1 < nsl;
    const int s = global_of(il);
#if QSC_FAIR_PRIO
    prio_level(3 - min(3, n));  // (uniform: the wave's n-th slice)
#endif
#if QSC_FIRST_WAIT
    // the first slice's reads land before the second slice's are issued: the launch's first
    // burst is then one slice per wave, not two
    if (n == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      STAMP(wg, 12);
    }
#endif
    QSC_DCHECK(s < nt * nsl && s_off[s] + (int64_t)s_width[s] * QSC_SLICE <= lk.dbg_ent[0]);
    slice_load(q, s_ent, s_width, s_off, more ? global_of(il1) : s, ln, S, mS, vS);
    float sv[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) sv[r] = c.sv[r];
    f2v own[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) own[j] = f2v{sv[2 * j], sv[2 * j + 1]} * splat2(own_scale);
    f2v accp[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) accp[j] = splat2(0.0f);
    f2v nll = splat2(0.0f);
    walk_halves<RP, E, KIND, LOG>(c.src, ln.ent, 2 * QSC_SLICE, c.j1, c.buf, own, Cl, El, lk,
                                  accp, nll);
    float acc[RP];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) {
      acc[2 * j] = accp[j].x;
      acc[2 * j + 1] = accp[j].y;
    }
    float a[RH], pv[RH], m[RH], v[RH];
#pragma unroll
    for (int j = 0; j < RH; ++j) {
      a[j] = half_sum_pick(acc[j], acc[RH + j]);
      pv[j] = swap_lo(sv[j], sv[RH + j]);
      m[j] = c.mv[j];
      v[j] = c.vv[j];
    }
    float nsq = adam_row_fast<RH>(pv, m, v, a, sc.coef, sc.as, ad.project_nonneg != 0);
    const int64_t blk = (int64_t)s * QSC_SLICE * RP;  // the slice's rows (uniform)
    st_row_wt<RH>(S + blk, ln.half, pv);
    st_row_wt<RH>(mS + blk, ln.half, m);
    st_row_wt<RH>(vS + blk, ln.half, v);
    st_row<RH>(Sl + (il * QSC_SLICE + p) * CP + h * RH, pv);  // the tile row, for the C-pass
    if constexpr (is_sr(KIND)) {
      float nv[RH];
#pragma unroll
      for (int j = 0; j < RH; ++j) nv[j] = -pv[j];
      st_row<RH>(Sl + (sr_off(PT) + il * QSC_SLICE + p) * CP + h * RH, nv);
    }
    nsq = wave_sum_dpp(nsq);
    if (lane == 0) part_nsq_s[s] = nsq;
    const float nll_w = wave_sum_dpp(nll.x + nll.y) * kLn2;
    if (lane == 0) part_nll_s[s] = nll_w;
    STAMP(wg, 5 + min(n, 8));  // end of the wave's n-th slice
    il = il1;
    ++n;
    return more;
  };
  // 3. C-pass units of the tile at the new S (cpass_tile_kernel steps 1, 3, 4).
  int u = w;
  V4 buf[kGroup];
  float cv[RP];
  int wi = 0, jb = 0, je = 0, js = 1, k = 0;
  const V4* src = nullptr;
  const uint32_t lo = (uint32_t)lane * (uint32_t)sizeof(V4);
  // unit uu: its list block and chunk range, the read-ahead of its first chunk group, its bin
  // and C column
  auto unit_begin = [&](int uu) {
    const int ks = uu / NP, part = uu - ks * NP;
    wi = t * nks + ks;
    const int W4 = c_width[wi] >> 2;
    const PartRange pr = part_range(W4, part, NP);
    jb = pr.j0;
    je = pr.j1;
    js = pr.js;
    src = reinterpret_cast<const V4*>(c_ent + c_off[wi]);
    QSC_DCHECK(c_off[wi] + (int64_t)c_width[wi] * 64 <= lk.dbg_ent[1]);
    load_group(src, lo, 64, jb, js, max(pr.j1 - 1, 0), buf);
    k = c_kmap[wi * 64 + lane];  // this lane's bin (count-sorted order)
    QSC_DCHECK(k >= 0 && k < Kp);
#pragma unroll
    for (int r = 0; r < RP; ++r) cv[r] = Cl[min(k, K - 1) * CP + r];  // C_i, as the S-step used
  };
  f2v cnll = splat2(0.0f);
  auto unit_walk = [&](f2v (&accp)[RP / 2]) {
    f2v own[RP / 2];
#pragma unroll
    for (int j = 0; j < RP / 2; ++j)
      own[j] = f2v{(2 * j < R && k < K) ? cv[2 * j] : 0.0f,
                   (2 * j + 1 < R && k < K) ? cv[2 * j + 1] : 0.0f} * splat2(own_scale);
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) accp[j] = splat2(0.0f);
    walk_groups<RP, E, KIND, LOG>(src, lo, 64, jb, je, js, buf, own, Sl, El, lk, accp, cnll);
  };
  auto to_pl = [&](const f2v (&accp)[RP / 2]) {
#pragma unroll
    for (int j = 0; j < RP / 2; ++j) {
      if (2 * j < R) Pl[((size_t)u * R + 2 * j) * 64 + lane] = accp[j].x;
      if (2 * j + 1 < R) Pl[((size_t)u * R + 2 * j + 1) * 64 + lane] = accp[j].y;
    }
  };

  // 2. S-step over the wave's slices (next slice's reads in flight; the two register sets
  //    alternate, as in spass_kernel)
  if (il < nsl) {
    SliceIn<RP, E, ADAM> nxt;
    const bool more = one_slice(cur, nxt);  // round 1 (peeled: its first-slice wait, n == 0)
    if (more)
      for (;;) {
        if (!one_slice(nxt, cur)) break;
        if (!one_slice(cur, nxt)) break;
      }
  }

  // the next launch's S-step scalars, by the oldest wave of block 0 (it has slack: its slices
  // are done long before the tile barrier)
  if (t == 0 && tidx == 0) adam_cache_store(acache, ad, step_s + 2);

  STAMP(wg, 2);
  if (u < U) unit_begin(u);
  __syncthreads();  // the whole S tile is in LDS
  STAMP(wg, 3);
  for (; u < U; u += NW) {
    f2v accp[RP / 2];
    unit_walk(accp);
    const float nll_w = wave_sum_dpp(cnll.x + cnll.y) * kLn2;
    cnll = splat2(0.0f);
    if (NP == 1) {
#pragma unroll
      for (int j = 0; j < RP / 2; ++j) {
        if (2 * j < R) slab[((int64_t)t * R + 2 * j) * Kp + k] = accp[j].x;
        if (2 * j + 1 < R) slab[((int64_t)t * R + 2 * j + 1) * Kp + k] = accp[j].y;
      }
      if (lane == 0) part_nll_c[wi] = nll_w;
    } else {
      to_pl(accp);
      if (lane == 0) Nl[u] = nll_w;
    }
    if (u + NW < U) unit_begin(u + NW);
  }
  STAMP(wg, 4);
  if (NP > 1) {
    __syncthreads();
    for (int i = tidx, j = 0; i < nks * R * 64; i += blockDim.x, ++j) {
      const int ks = i / (R * 64), rl = i - ks * (R * 64);
      const float* pp0 = Pl + (size_t)ks * NP * R * 64 + rl;
      float acc = pp0[0];
      for (int pp = 1; pp < NP; ++pp) acc += pp0[(size_t)pp * R * 64];
      const int r = rl >> 6, l = rl & 63;
#if QSC_KMAP_PF
      const int kk = j == 0 ? km_pf[0] : j == 1 ? km_pf[1] : c_kmap[((int64_t)t * nks + ks) * 64 + l];
#else
      const int kk = c_kmap[((int64_t)t * nks + ks) * 64 + l];
#endif
      slab[((int64_t)t * R + r) * Kp + kk] = acc;
    }
    for (int ks = tidx; ks < nks; ks += blockDim.x) {
      float acc = Nl[ks * NP];
      for (int pp = 1; pp < NP; ++pp) acc += Nl[ks * NP + pp];
      part_nll_c[t * nks + ks] = acc;
    }
  }
  STAMP(wg, kStampLast);
  RSTAMP(wg, 29);
}

template <int RP, typename E, int KIND, bool LOG>
__global__ void __launch_bounds__(FusedBlock<RP>::v, FusedBlock<RP>::wpe)
scfused_kernel(QSC_SCF_KPARAMS) {
  scfused_tile<RP, E, KIND, LOG>(QSC_SCF_ARGS, (int)blockIdx.x, (int)gridDim.x, threadIdx.x);
}

// LDS bytes of scfused_kernel
size_t scfused_lds(int PT, int R, int K, int nks, int NP, bool sr) {
  const size_t U = (size_t)nks * NP;
  return 32 + tfloats(K, R, sr) * 4 + 256 * 8 + tfloats(PT, R, sr) * 4 +
         (NP > 1 ? U * R * 64 * 4 : 0) + std::max<size_t>(U, 16) * 4;
}

// The C-pass tile partition of a layout: NP parts per bin list, up to 16 waves per tile, while
// a part keeps >= QSC_CPART_MIN_CHUNKS 4-entry chunks and, at the signed-row size (the same NP
// for both row formats), the tile form's LDS fits and so does the fused launch's where it can
// fit at all; true when the tile form applies (>= 4 units, LDS fits at the layout's own row
// format `sr`)
// rank 16: units (k-slices x parts) per tile at most -- 8, one per wave of the 8-wave
// workgroups: c4k K-slab C-pass 24.8 us at 16 units (two per wave), 22.6 us at 8, 22.7 us with
// 12 units on 12-wave workgroups (profiles/r06/r16/ab_r16_units_waves.log)
#ifndef QSC_R16_UNITS
#define QSC_R16_UNITS 8
#endif
static bool tile_parts(const qsc_obs_desc* d, int R, bool sr, int* np) {
  const int nks = d->nks;
  const int maxu = R > 8 ? QSC_R16_UNITS : QSC_CTILE_MAXW;
  int NP = nks >= maxu ? 1 : maxu / nks;
  const double chunks = (double)d->nnz / ((double)d->ntiles * d->K) / 4.0;
  const bool fused = scfused_lds(d->PT, R, d->K, nks, 1, true) <= 160 * 1024;
  while (NP > 1 && (chunks / NP < QSC_CPART_MIN_CHUNKS ||
                    cpass_tile_lds(d->PT, R, nks, NP, true) > 160 * 1024 ||
                    (fused && scfused_lds(d->PT, R, d->K, nks, NP, true) > 160 * 1024)))
    --NP;
  *np = NP;
  return QSC_CPASS_TILE && nks * NP >= 4 && cpass_tile_lds(d->PT, R, nks, NP, sr) <= 160 * 1024;
}

// ---------------------------------------------------------------------------------------
// The fixed order of the scalar partials -- the S-passes' per-slice NLL and ||S||^2
// (part_nll_s, part_nsq_s) and the C-passes' per-(tile, k-slice) NLL (part_nll_c) -- which every
// form settles (cfinish's book-keeping block, state_flush: both 1024-thread blocks), so that the
// solver forms agree bit for bit: thread i sums items i, i + 1024, i + 2048, ... in order (every
// load of a batch of 8 issued before the sums: one memory round trip at C3's 8192 slices instead
// of a dependent chain per tile); then each wave's xor butterfly (wave_sum) and the 16 wave sums
// in wave order; every sum from +0.
// ---------------------------------------------------------------------------------------
struct Canon {
  float nll_s, nsq_s, nll_c;
};

__device__ __forceinline__ float canon_part(const float* __restrict__ x, int n, int tid, int nb) {
  float a = 0.0f;
  if (!x) return a;
  for (int i0 = tid; i0 < n; i0 += 8 * nb) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[min(i0 + j * nb, n - 1)];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i0 + j * nb < n) a += v[j];
  }
  return a;
}

// The three totals over nslices S-pass items and nc C-pass items; sh: LDS [3][nb / 64] floats.
// Result valid in thread 0.
__device__ Canon canon_totals(const float* __restrict__ nll_s, const float* __restrict__ nsq_s,
                              const float* __restrict__ nll_c, int nslices, int nc, float* sh) {
  const int nb = blockDim.x, tid = threadIdx.x, nw = nb >> 6;
  float a = canon_part(nll_s, nslices, tid, nb);
  float b = canon_part(nsq_s, nslices, tid, nb);
  float c = canon_part(nll_c, nc, tid, nb);
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  if ((tid & 63) == 0) {
    sh[tid >> 6] = a;
    sh[nw + (tid >> 6)] = b;
    sh[2 * nw + (tid >> 6)] = c;
  }
  __syncthreads();
  Canon r{0.0f, 0.0f, 0.0f};
  if (tid == 0)
    for (int w = 0; w < nw; ++w) {
      r.nll_s += sh[w];
      r.nsq_s += sh[nw + w];
      r.nll_c += sh[2 * nw + w];
    }
  return r;
}

// book-keeping shared by cfinish (block 0) and state_flush: settle a pending S-pass
__device__ void settle_s(qsc_state* __restrict__ st, const float* __restrict__ part_nll_s,
                         const float* __restrict__ part_nsq_s, int nslices, float* hist,
                         int hist_cap, float* sh) {
  const int pend = st->pending;  // uniform read (all threads)
  if (!(pend & (QSC_PEND_SNLL | QSC_PEND_SUPD))) return;
  const Canon c = canon_totals(part_nll_s, (pend & QSC_PEND_SUPD) ? part_nsq_s : nullptr, nullptr,
                               nslices, 0, sh);
  if (threadIdx.x == 0) {
    const int it = st->iter - 1;
    st->nll_s = c.nll_s;
    if (hist && it >= 0 && it < hist_cap) {
      hist[4 * it + 0] = st->nll_c;
      hist[4 * it + 1] = c.nll_s;
      hist[4 * it + 2] = st->normsq_c;
      hist[4 * it + 3] = st->normsq_s_prev;
    }
    if (pend & QSC_PEND_SUPD) {
      st->normsq_s = c.nsq_s;
      st->step_s += 1;
    }
    st->pending = pend & ~(QSC_PEND_SNLL | QSC_PEND_SUPD);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------
// C finish: fixed-order slab reduction (+ fused regulariser / Adam / projection)
// ---------------------------------------------------------------------------------------
#define QSC_CF_PARAMS                                                                          \
  const float *__restrict__ slab, int ntiles, int nks, int R, int K, float *C, int mode,         \
      float *__restrict__ dC, float *__restrict__ mC, float *__restrict__ vC, qsc_adam ad,       \
      float lambda_c, const float *__restrict__ normsq_ext, const float *__restrict__ cnsq,      \
      qsc_state *__restrict__ st, const float *__restrict__ part_nll_c, int npart_c,             \
      const float *__restrict__ part_nll_s, const float *__restrict__ part_nsq_s, int nslices,   \
      float *__restrict__ hist, int hist_cap, AdamCache *__restrict__ acache
#define QSC_CF_ARGS                                                                           \
  slab, ntiles, nks, R, K, C, mode, dC, mC, vC, ad, lambda_c, normsq_ext, cnsq, st, part_nll_c,  \
      npart_c, part_nll_s, part_nsq_s, nslices, hist, hist_cap, acache
constexpr int kFWaves = kFBlock / 64;

// the C-finish tile sum of the VF virtual waves vw = wave + f NWp (f < VF) of this wave: each
// virtual wave's column partial sums its tiles vw, vw + 16, ... in order; sixteen loads in
// flight per lane (16 / VF tiles of each virtual wave per batch), so a 4..15-wave workgroup
// holds no more registers for it than the 16-wave one
template <int VF>
__device__ __forceinline__ void cfin_tile_sum(float (*red)[64], const float* col,
                                              const int64_t tstride, const int ntiles,
                                              const int wave, const int NWp, const int lane) {
  // NGB: groups of 16 NW tiles per batch.  Two in the standalone C-finish (32 loads in flight)
  // made it slower, 3.26 -> 4.6 us at C3 (profiles/r04/fin_small_wg/ab_c3_grouped_tickets.log)
  constexpr int NW = kFWaves, JB = 16 / VF, NGB = 1;
  float a[VF];
#pragma unroll
  for (int f = 0; f < VF; ++f) a[f] = 0.0f;
  for (int tg = 0; tg < ntiles; tg += NGB * 16 * NW) {
    for (int jb = 0; jb < 16; jb += JB) {
      float v[NGB][VF][JB];
#pragma unroll
      for (int gb = 0; gb < NGB; ++gb)
#pragma unroll
        for (int f = 0; f < VF; ++f) {
          const int vw = wave + f * NWp;
#pragma unroll
          for (int j = 0; j < JB; ++j) {
            const int tt = tg + gb * 16 * NW + vw + (jb + j) * NW;
            v[gb][f][j] =
                vw < NW ? col[(int64_t)min(tt, ntiles - 1) * tstride] : 0.0f;
          }
        }
#pragma unroll
      for (int gb = 0; gb < NGB; ++gb)
#pragma unroll
        for (int f = 0; f < VF; ++f) {
          const int vw = wave + f * NWp;
#pragma unroll
          for (int j = 0; j < JB; ++j)
            if (vw < NW && tg + gb * 16 * NW + vw + (jb + j) * NW < ntiles) a[f] += v[gb][f][j];
        }
    }
  }
#pragma unroll
  for (int f = 0; f < VF; ++f)
    if (wave + f * NWp < NW) red[wave + f * NWp][lane] = a[f];
}

// C-finish work item vb of R*nks + 2 (cfinish_kernel: vb = the workgroup), with its LDS scratch
// passed in: per (r, 64-bin slice) column block the 16 waves' partials (wave w: tiles w, w + 16,
// ... in order -- the canonical tile groups, canon_totals) summed in wave order; item R*nks the
// book-keeping (canon_totals), item R*nks + 1 the next C-step's Adam scalars.
__device__ __forceinline__ void cfinish_vb(const int vb, float (*red)[64], Scalars& sc, float* sh,
                                           QSC_CF_PARAMS) {
  constexpr int NW = kFWaves;
  const int NWp = NW;
  const int Kp = nks * 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;

  // ||C||^2 of the C this step differentiates: written by the C-pass (C is read-only there),
  // or the caller's global value (K-slab); never re-read here, where blocks overwrite C
  const float nsq = normsq_ext ? *normsq_ext : *cnsq;

  if (vb == R * nks + 1) {
    // the next C-step's Adam scalars (the next S-pass settles step_c + 1 in between)
    if (mode == 1 && threadIdx.x == 0) adam_cache_store(acache, ad, st->step_c + 2);
    return;
  }
  if (vb == R * nks) {
    // book-keeping block: settle the S-pass partials (settle_s) and total the C-pass NLL, in
    // the canonical order (canon_totals)
    const int pend = st->pending;
    const bool settle = (pend & (QSC_PEND_SNLL | QSC_PEND_SUPD)) != 0;
    const bool supd = (pend & QSC_PEND_SUPD) != 0;
    const Canon cs = canon_totals(settle ? part_nll_s : nullptr, supd ? part_nsq_s : nullptr,
                                  part_nll_c, nslices, npart_c, sh);
    if (threadIdx.x == 0) {
      int pnd = pend;
      if (settle) {  // settle_s, thread-0 part
        const int it = st->iter - 1;
        st->nll_s = cs.nll_s;
        if (hist && it >= 0 && it < hist_cap) {
          hist[4 * it + 0] = st->nll_c;
          hist[4 * it + 1] = cs.nll_s;
          hist[4 * it + 2] = st->normsq_c;
          hist[4 * it + 3] = st->normsq_s_prev;
        }
        if (supd) {
          st->normsq_s = cs.nsq_s;
          st->step_s += 1;
        }
        pnd = pend & ~(QSC_PEND_SNLL | QSC_PEND_SUPD);
        st->pending = pnd;
      }
      st->nll_c = cs.nll_c;
      if (mode == 1) {
        st->normsq_c = nsq;
        st->pending = pnd | QSC_PEND_C;
      }
      if (mode == 2) dC[(int64_t)R * K] = st->normsq_s;  // this shard's ||S||^2 (IJ-slab)
    }
    return;
  }

  const int r = vb / nks, ks = vb - r * nks;
  const int k = ks * 64 + lane;
  // wave 0 reads its C / moments ahead of the tile sum (one HBM round trip instead of two)
  float p0 = 0.0f, m0 = 0.0f, v0 = 0.0f;
  if (mode == 1 && wave == 0 && k < K) {
    const int64_t i = (int64_t)r * K + k;
    p0 = C[i];
    m0 = mC[i];
    v0 = vC[i];
  }
  if (threadIdx.x == 0 && mode == 1) {
    const AdamCache a0 = acache[0], a1 = acache[1];  // both slots: no dependent read on step_c
    const int step = st->step_c + 1;
    const float nrm = sqrtf(nsq);
    sc.coef = nrm > 0.0f ? lambda_c / nrm : 0.0f;
    sc.as = adam_scalars_cached((step & 1) ? a1 : a0, ad, step);
  }
  // tile sum: (virtual) wave w takes tiles w, w+16, ...; sixteen independent loads in flight
  const float* col = slab + (int64_t)r * Kp + k;
  const int64_t tstride = (int64_t)R * Kp;
  cfin_tile_sum<1>(red, col, tstride, ntiles, wave, NWp, lane);
  __syncthreads();
  if (wave == 0 && k < K) {
    float g = red[0][lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) g += red[w][lane];
    const int64_t i = (int64_t)r * K + k;
    if (mode == 1) {
      float p = p0, m = m0, v = v0;
      g = __fadd_rn(g, __fmul_rn(p, sc.coef));
      adam_elem(p, m, v, g, ad, sc.as);
      C[i] = p;
      mC[i] = m;
      vC[i] = v;
    } else {
      dC[i] = g;  // modes 0 and 2
    }
  }
}

__global__ void __launch_bounds__(kFBlock) cfinish_kernel(QSC_CF_PARAMS) {
  __shared__ float red[kFWaves][64];
  __shared__ Scalars sc;
  __shared__ float sh[3 * kFWaves];
  cfinish_vb((int)blockIdx.x, red, sc, sh, QSC_CF_ARGS);
}


// ---------------------------------------------------------------------------------------
// C update from an externally reduced gradient g [R][K] (IJ-slab sharding, after the RCCL
// all-reduce of the per-shard dC): g + lambda_c C/||C||, Adam, C >= 0; the same state
// protocol as qsc_cfinish mode 1.  normsq_s_ext (nullable): the all-reduced ||S||^2, stored as
// the S-pass's regulariser norm.
__global__ void __launch_bounds__(kFBlock) cupdate_kernel(
    int R, int K, float* __restrict__ C, float* __restrict__ mC, float* __restrict__ vC,
    const float* __restrict__ g, qsc_adam ad, float lambda_c,
    const float* __restrict__ normsq_s_ext, qsc_state* __restrict__ st) {
  constexpr int NW = kFBlock / 64;
  __shared__ float shn[NW];
  __shared__ Scalars sc;
  const int n = R * K;
  const float nsq = cnorm_sq(C, n, shn);
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(nsq);
    sc.coef = nrm > 0.0f ? lambda_c / nrm : 0.0f;
    sc.as = adam_scalars(ad, st->step_c + 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float p = C[i], m = mC[i], v = vC[i];
    const float gg = __fadd_rn(g[i], __fmul_rn(p, sc.coef));
    adam_elem(p, m, v, gg, ad, sc.as);
    C[i] = p;
    mC[i] = m;
    vC[i] = v;
  }
  if (threadIdx.x == 0) {
    st->normsq_c = nsq;
    st->pending |= QSC_PEND_C;
    if (normsq_s_ext) st->normsq_s = *normsq_s_ext;
  }
}

__global__ void __launch_bounds__(1024) flush_kernel(qsc_state* __restrict__ st,
                                                     const float* __restrict__ part_nll_s,
                                                     const float* __restrict__ part_nsq_s,
                                                     int ntiles, int nslices,
                                                     float* __restrict__ hist, int hist_cap) {
  __shared__ float sh[3 * 16];
  settle_s(st, part_nll_s, part_nsq_s, nslices, hist, hist_cap, sh);
  if (threadIdx.x == 0 && (st->pending & QSC_PEND_C)) {
    st->step_c += 1;
    st->pending &= ~QSC_PEND_C;
  }
}

// S update from an all-reduced gradient (K-slab): the S-pass's lane mapping (32 positions per
// wave, lane half h owns the row elements [h*RP/2, (h+1)*RP/2)) and its Adam
template <int RP>
__global__ void __launch_bounds__(kSBlock) supdate_kernel(
    int nslices, float* __restrict__ S, float* __restrict__ mS, float* __restrict__ vS,
    const float* __restrict__ gsrc, qsc_adam ad, float lambda_s, qsc_state* __restrict__ st,
    float* __restrict__ part_nsq) {
  constexpr int RH = RP / 2;
  __shared__ Scalars sc;
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(st->normsq_s);
    sc.coef = nrm > 0.0f ? lambda_s / nrm : 0.0f;
    sc.as = adam_scalars(ad, st->step_s + 1);
    if (blockIdx.x == 0) st->pending |= QSC_PEND_SUPD;  // normsq_s / step_s settled later
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * kSWaves + wave;
  if (s >= nslices) return;
  const int64_t o = ((int64_t)s * QSC_SLICE + (lane & (QSC_SLICE - 1))) * RP + (lane >> 5) * RH;
  float p[RH], m[RH], v[RH], g[RH];
  ld_row<RH>(S + o, p);
  ld_row<RH>(mS + o, m);
  ld_row<RH>(vS + o, v);
  ld_row<RH>(gsrc + o, g);
  // the fused S-pass's update (no projection)
  float nsq = adam_row_fast<RH>(p, m, v, g, sc.coef, sc.as, ad.project_nonneg != 0);
  st_row<RH>(S + o, p);
  st_row<RH>(mS + o, m);
  st_row<RH>(vS + o, v);
  nsq = wave_sum(nsq);
  if (lane == 0) part_nsq[s] = nsq;
}

// K-slab S update on this rank's shard of slices [s0, s0 + gridDim slices) with the shard's
// reduce-scattered gradient g_own (rows of slice s0 first): the same lane mapping, Adam and
// per-slice ||S_new||^2 partial as supdate_kernel, for the owned rows only
template <int RP>
__global__ void __launch_bounds__(kSBlock) supdate_slices_kernel(
    int s0, int s1, float* __restrict__ S, float* __restrict__ mS, float* __restrict__ vS,
    const float* __restrict__ g_own, qsc_adam ad, float lambda_s, qsc_state* __restrict__ st,
    float* __restrict__ part_nsq) {
  constexpr int RH = RP / 2;
  __shared__ Scalars sc;
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(st->normsq_s);
    sc.coef = nrm > 0.0f ? lambda_s / nrm : 0.0f;
    sc.as = adam_scalars(ad, st->step_s + 1);
    if (blockIdx.x == 0) st->pending |= QSC_PEND_SUPD;  // normsq_s / step_s settled later
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = s0 + blockIdx.x * kSWaves + wave;
  if (s >= s1) return;
  const int64_t lo = ((int64_t)(lane & (QSC_SLICE - 1))) * RP + (lane >> 5) * RH;
  const int64_t o = (int64_t)s * QSC_SLICE * RP + lo;
  const int64_t og = (int64_t)(s - s0) * QSC_SLICE * RP + lo;
  float p[RH], m[RH], v[RH], g[RH];
  ld_row<RH>(S + o, p);
  ld_row<RH>(mS + o, m);
  ld_row<RH>(vS + o, v);
  ld_row<RH>(g_own + og, g);
  float nsq = adam_row_fast<RH>(p, m, v, g, sc.coef, sc.as, ad.project_nonneg != 0);
  st_row<RH>(S + o, p);
  st_row<RH>(mS + o, m);
  st_row<RH>(vS + o, v);
  nsq = wave_sum(nsq);
  if (lane == 0) part_nsq[s] = nsq;
}

// Per-slice ||S||^2 partials of a replicated S, bit-identical to the ones supdate_kernel /
// supdate_slices_kernel compute from the same rows (same lane mapping, the same fma chain over
// the lane's half row, the same wave sum): after the K-slab all-gather every rank holds every
// slice's partial without exchanging them
template <int RP>
__global__ void __launch_bounds__(kSBlock) slice_nsq_kernel(int nslices,
                                                            const float* __restrict__ S,
                                                            float* __restrict__ part_nsq) {
  constexpr int RH = RP / 2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * kSWaves + wave;
  if (s >= nslices) return;
  const int64_t o = ((int64_t)s * QSC_SLICE + (lane & (QSC_SLICE - 1))) * RP + (lane >> 5) * RH;
  float p[RH];
  ld_row<RH>(S + o, p);
  float nsq = 0.0f;
#pragma unroll
  for (int j = 0; j < RH; ++j) nsq = __builtin_fmaf(p[j], p[j], nsq);
  nsq = wave_sum(nsq);
  if (lane == 0) part_nsq[s] = nsq;
}

__global__ void state_init_kernel(qsc_state* st, const double* nsq_part, int nparts) {
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < nparts; ++i) s += nsq_part[i];
    qsc_state z{};
    z.normsq_s = (float)s;
    z.normsq_s_prev = (float)s;
    *st = z;
  }
}

__global__ void __launch_bounds__(kSBlock) nsq_part_kernel(const float* __restrict__ x, int64_t n,
                                                           double* __restrict__ part) {
  __shared__ double sh[kSWaves];
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    s += v * v;
  }
  const double r = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

__global__ void __launch_bounds__(1024) sumsq_small_kernel(const float* __restrict__ x, int n,
                                                           float* __restrict__ out) {
  __shared__ float sh[16];
  const float r = cnorm_sq(x, n, sh);  // the C-pass's order
  if (threadIdx.x == 0) *out = r;
}

// Adam on a flat parameter buffer (the generator / DIP solver's decoder weights or latent Z,
// torch.optim.Adam's update bit for bit: adam_elem) at step = the state's S-pass counter, so one
// captured hipGraph replays every iteration's step (qsc_adam_flat)
__global__ void __launch_bounds__(256) adam_flat_kernel(float* __restrict__ p,
                                                        float* __restrict__ m,
                                                        float* __restrict__ v,
                                                        const float* __restrict__ g, int64_t n,
                                                        qsc_adam ad,
                                                        const qsc_state* __restrict__ st) {
  __shared__ AdamScalars sc;
  if (threadIdx.x == 0) sc = adam_scalars(ad, st->iter);
  __syncthreads();
  const AdamScalars s = sc;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(pp, mm, vv, g[i], ad, s);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

__global__ void selftest_erf_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = erff(x[i]);
  out[n + i] = erf_fast(x[i]);
}

// ---- workspace layout ----
struct PassWs {
  float* slab;      // ntiles * R * Kp
  float* cnll;      // ntiles * nks
  float* snll;      // nslices
  float* snsq;      // nslices
  double* init;     // 256
  int* sched;       // S-pass queue counters [kSchedQ] + finished-wave counter (zero between launches)
  float* cnsq;      // ||C||^2 of the C the last C-pass read (written by the C-pass)
  AdamCache* acache;  // [0..1] S-side, [2..3] C-side step scalars (adam_scalars_cached)
};

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

PassWs carve(const qsc_obs_desc* d, int R, void* ws) {
  char* w = (char*)ws;
  PassWs p;
  const int64_t Kp = (int64_t)d->nks * 64;
  p.slab = (float*)w;
  w += al((size_t)d->ntiles * R * Kp * 4);
  p.cnll = (float*)w;
  w += al((size_t)d->ntiles * d->nks * 4);
  p.snll = (float*)w;
  w += al((size_t)(d->Pp / QSC_SLICE) * 4);
  p.snsq = (float*)w;
  w += al((size_t)(d->Pp / QSC_SLICE) * 4);
  p.init = (double*)w;
  w += al(256 * 8);
  p.sched = (int*)w;
  w += al((kSchedQ + 1) * 4);
  p.cnsq = (float*)w;
  w += al(4);
  p.acache = (AdamCache*)w;
  w += al(4 * sizeof(AdamCache));
  return p;
}

size_t ws_bytes_for(const qsc_obs_desc* d, int R) {
  const int64_t Kp = (int64_t)d->nks * 64;
  return al((size_t)d->ntiles * R * Kp * 4) + al((size_t)d->ntiles * d->nks * 4) +
         2 * al((size_t)(d->Pp / QSC_SLICE) * 4) + al(256 * 8) + al((kSchedQ + 1) * 4) + al(4) +
         al(4 * sizeof(AdamCache));
}

bool desc_ok(const qsc_obs_desc* d) {
  return d && d->K >= 1 && d->P >= 1 && d->Pp >= d->P && (d->Pp % 64) == 0 && d->PT >= 64 &&
         (d->PT % 64) == 0 && d->ntiles * d->PT == d->Pp && d->nks * 64 >= d->K &&
         d->nbins >= 1;
}

int rp_of(int R) { return R <= 4 ? 4 : (R <= 8 ? 8 : 16); }

// linear model edges pre-divided by a for the scaled entry form (lik_grad2)
void scale_edges(Edges* E, int nbins, float a) {
  for (int c = 0; c < nbins; ++c)
    E->e[c] = make_float2((float)((double)E->e[c].x / a), (float)((double)E->e[c].y / a));
}

// the QSC_DEBUG bounds of a launch (Lik::dbg_*): gather-table rows and entry counts
void set_dbg(Lik& lk, const qsc_obs_desc* d, bool sr) {
  lk.dbg_rows[0] = sr ? sr_rows(d->K) : d->K;
  lk.dbg_rows[1] = sr ? sr_rows(d->PT) : d->PT;
  lk.dbg_ent[0] = d->s_entries;
  lk.dbg_ent[1] = d->c_entries;
}

// compute units of the current device (cached per device id)
int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// resident S-pass workgroups per CU (persistent grid); RP=16 needs twice the registers
#ifndef QSC_SPASS_BPC
#define QSC_SPASS_BPC 2
#endif

size_t cpass_lds(const qsc_obs_desc* d, int R, bool sr) {
  return tfloats(d->PT, R, sr) * 4 + 2 * 256 * 4 + (size_t)kCParts * R * 64 * 4 + kCParts * 4;
}
size_t spass_lds(const qsc_obs_desc* d, int R, bool sr) {
  return 32 + tfloats(d->K, R, sr) * 4 + (size_t)d->nbins * 8;
}
int spass_bpc(int RP) { return RP > 8 ? 2 : RP == 8 ? QSC_SPASS_BPC8 : QSC_SPASS_BPC; }

}  // namespace

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

// dispatch over (RP, entry type, likelihood kind, log) for a kernel template K<RP,E,KIND,LOG,...>
#define QSC_DISPATCH_RP(LAUNCH, KD, LG)                                                  \
  do {                                                                                   \
    if (d->wide) {                                                                       \
      if (RP == 4) LAUNCH(4, uint32_t, KD, LG);                                          \
      else if (RP == 8) LAUNCH(8, uint32_t, KD, LG);                                     \
      else LAUNCH(16, uint32_t, KD, LG);                                                 \
    } else {                                                                             \
      if (RP == 4) LAUNCH(4, uint16_t, KD, LG);                                          \
      else if (RP == 8) LAUNCH(8, uint16_t, KD, LG);                                     \
      else LAUNCH(16, uint16_t, KD, LG);                                                 \
    }                                                                                    \
  } while (0)
// signed-row layouts (rowfmt 1) are narrow and one-bit only
#define QSC_DISPATCH_RP_NARROW(LAUNCH, KD, LG)                                           \
  do {                                                                                   \
    if (RP == 4) LAUNCH(4, uint16_t, KD, LG);                                            \
    else if (RP == 8) LAUNCH(8, uint16_t, KD, LG);                                       \
    else LAUNCH(16, uint16_t, KD, LG);                                                   \
  } while (0)
#ifdef QSC_DEV_ONE_VARIANT  // (ISA work: only the signed-row instantiation of rank QSC_DEV_ONE_VARIANT)
#define QSC_DISPATCH_PASS(LAUNCH)                   \
  do {                                              \
    (void)kind;                                     \
    if (sr && RP == QSC_DEV_ONE_VARIANT) LAUNCH(QSC_DEV_ONE_VARIANT, uint16_t, LIK_ONEBIT_SR, false); \
    else return QSC_EUNSUPPORTED;                   \
  } while (0)
#else
#define QSC_DISPATCH_PASS(LAUNCH)                                                        \
  do {                                                                                   \
    if (sr) QSC_DISPATCH_RP_NARROW(LAUNCH, LIK_ONEBIT_SR, false);                        \
    else if (kind == LIK_ONEBIT) QSC_DISPATCH_RP(LAUNCH, LIK_ONEBIT, false);             \
    else if (kind == LIK_SQUARED && m->log_model) QSC_DISPATCH_RP(LAUNCH, LIK_SQUARED, true); \
    else if (kind == LIK_SQUARED) QSC_DISPATCH_RP(LAUNCH, LIK_SQUARED, false);           \
    else if (m->log_model) QSC_DISPATCH_RP(LAUNCH, LIK_GENERAL, true);                   \
    else QSC_DISPATCH_RP(LAUNCH, LIK_GENERAL, false);                                    \
  } while (0)
#endif

static bool rowfmt_ok(const qsc_obs_desc* d, int R, int kind);

extern "C" {

QSC_API size_t qsc_pass_workspace_bytes(const qsc_obs_desc* d, int32_t R) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R) return 0;
  return ws_bytes_for(d, R);
}

QSC_API int qsc_state_init(qsc_state* st, const float* S, int32_t R, int32_t Pp, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!st || R < 1 || R > QSC_MAX_R || Pp < 1 || !ws || ws_bytes < 256 * sizeof(double))
    return QSC_EINVAL;
  double* part = (double*)ws;
  const int nb = 256;
  if (S) {
    hipLaunchKernelGGL(nsq_part_kernel, dim3(nb), dim3(kSBlock), 0, STREAM(stream), S,
                       (int64_t)rp_of(R) * Pp, part);  // [Pp][RP], padding rows are zero
    QSC_CHECK_LAUNCH();
  } else {
    QSC_TRY(hipMemsetAsync(part, 0, nb * sizeof(double), STREAM(stream)));
  }
  hipLaunchKernelGGL(state_init_kernel, dim3(1), dim3(64), 0, STREAM(stream), st, part, nb);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

static int spass_impl(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                      const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                      const float* C, int32_t mode, float* dS, float* mS, float* vS,
                      const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                      size_t ws_bytes, void* stream, int ck, int nck);

QSC_API int qsc_spass(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                      const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                      const float* C, int32_t mode, float* dS, float* mS, float* vS,
                      const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                      size_t ws_bytes, void* stream) {
  return spass_impl(d, s_entries, s_width, s_off, m, R, S, C, mode, dS, mS, vS, adam, lambda_s,
                    st, ws, ws_bytes, stream, 0, 0);
}

QSC_API int qsc_spass_kslab(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                            const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                            const float* C, float* dS_rs, int32_t chunk_slices, int32_t nranks,
                            qsc_state* st, void* ws, size_t ws_bytes, void* stream) {
  const int nslices = d ? d->Pp / QSC_SLICE : 0;
  if (!d || chunk_slices < 1 || nranks < 1 || (int64_t)chunk_slices * nranks < nslices ||
      !dS_rs)
    return QSC_EINVAL;
  return spass_impl(d, s_entries, s_width, s_off, m, R, S, C, 0, dS_rs, nullptr, nullptr,
                    nullptr, 0.0f, st, ws, ws_bytes, stream, chunk_slices, nranks);
}

static int spass_impl(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                      const int64_t* s_off, const qsc_model* m, int32_t R, float* S,
                      const float* C, int32_t mode, float* dS, float* mS, float* vS,
                      const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                      size_t ws_bytes, void* stream, int ck, int nck) {
  if (!desc_ok(d) || !m || m->nbounds - 1 != d->nbins || R < 1 || R > QSC_MAX_R || !S || !C ||
      !s_width || !s_off || (d->s_entries > 0 && !s_entries) || !ws || !st ||
      ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  if (mode == 0 && !dS) return QSC_EINVAL;
  if (mode == 1 && (!mS || !vS || !adam)) return QSC_EINVAL;
  if (mode != 0 && mode != 1) return QSC_EINVAL;
  const int RP = rp_of(R);
  const int kind = lik_kind(m);
  const bool sr = d->rowfmt == 1;
  if (!rowfmt_ok(d, R, kind)) return QSC_EINVAL;
  const size_t shm = spass_lds(d, R, sr);
  if (shm > 160 * 1024) return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  Edges E;
  make_edges(m, &E);
  Lik lk = make_lik(m);
  set_dbg(lk, d, sr);
  if (kind == LIK_SQUARED)
    make_sq_targets(m, &E);
  else if (!m->log_model)
    scale_edges(&E, m->nbounds - 1, lk.a);
  const int nslices = d->Pp / QSC_SLICE;
  const int bpc = spass_bpc(RP);
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(nslices, kSWaves), (int64_t)cu_count() * bpc));
  qsc_adam ad{};
  if (adam) ad = *adam;
  hipStream_t s = STREAM(stream);
#define SPASS_LAUNCH(RPV, ET, KD, LG)                                                          \
  do {                                                                                         \
    if (mode == 1)                                                                             \
      hipLaunchKernelGGL((spass_kernel<RPV, ET, KD, LG, true>), grid, dim3(kSBlock), shm, s,   \
                         (const ET*)s_entries, s_width, s_off, nslices, lk, E, d->nbins, R,    \
                         d->K, d->Pp, S, C, dS, mS, vS, ad, lambda_s, st, w.snll, w.snsq,       \
                         w.sched, w.acache, 0, 0);                                             \
    else                                                                                       \
      hipLaunchKernelGGL((spass_kernel<RPV, ET, KD, LG, false>), grid, dim3(kSBlock), shm, s,  \
                         (const ET*)s_entries, s_width, s_off, nslices, lk, E, d->nbins, R,    \
                         d->K, d->Pp, S, C, dS, mS, vS, ad, lambda_s, st, w.snll, w.snsq,       \
                         w.sched, w.acache, ck, nck);                                          \
  } while (0)
  QSC_DISPATCH_PASS(SPASS_LAUNCH);
#undef SPASS_LAUNCH
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

static int cpass_impl(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                      const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m, int32_t R,
                      const float* S, const float* C, void* ws, size_t ws_bytes, void* stream,
                      bool nsq);

QSC_API int qsc_cpass(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                      const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m, int32_t R,
                      const float* S, const float* C, void* ws, size_t ws_bytes, void* stream) {
  return cpass_impl(d, c_entries, c_width, c_off, c_kmap, m, R, S, C, ws, ws_bytes, stream,
                    false);
}

QSC_API int qsc_cpass_nsq(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                          const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m,
                          int32_t R, const float* S, const float* C, void* ws, size_t ws_bytes,
                          void* stream) {
  return cpass_impl(d, c_entries, c_width, c_off, c_kmap, m, R, S, C, ws, ws_bytes, stream,
                    true);
}


QSC_API int64_t qsc_pass_cnsq_offset(const qsc_obs_desc* d, int32_t R) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R) return -1;
  const uintptr_t base = 4096;  // any aligned address: the carve is base-relative
  return (int64_t)(reinterpret_cast<uintptr_t>(carve(d, R, reinterpret_cast<void*>(base)).cnsq) -
                   base);
}

static int cpass_impl(const qsc_obs_desc* d, const void* c_entries, const int32_t* c_width,
                      const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m, int32_t R,
                      const float* S, const float* C, void* ws, size_t ws_bytes, void* stream,
                      bool nsq) {
  if (!desc_ok(d) || !m || m->nbounds - 1 != d->nbins || R < 1 || R > QSC_MAX_R || !S || !C ||
      !c_width || !c_off || !c_kmap || (d->c_entries > 0 && !c_entries) || !ws ||
      ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  const int RP = rp_of(R);
  const int kind = lik_kind(m);
  const bool sr = d->rowfmt == 1;
  if (!rowfmt_ok(d, R, kind)) return QSC_EINVAL;
  const size_t shm = cpass_lds(d, R, sr);
  PassWs w = carve(d, R, ws);
  Edges E;
  make_edges(m, &E);
  Lik lk = make_lik(m);
  set_dbg(lk, d, sr);
  if (kind == LIK_SQUARED)
    make_sq_targets(m, &E);
  else if (!m->log_model)
    scale_edges(&E, m->nbounds - 1, lk.a);
  hipStream_t s = STREAM(stream);
  if (QSC_CPASS_TILE) {
    // tile form: up to 16 waves per tile, the partition of tile_parts
    const int nks = d->nks;
    int NP = 1;
    const bool tile = tile_parts(d, R, sr, &NP);
    const int U = nks * NP;
    size_t tshm = cpass_tile_lds(d->PT, R, nks, NP, sr);
    if (tile) {
      const dim3 tb((unsigned)(64 * std::min(U, RP > 8 ? QSC_CTILE_W16 : QSC_CTILE_MAXW)));
      // C^T staged in LDS when it fits next to the tile and in the threads' registers (kCT = 4
      // floats each): the units' C columns then come from LDS, not from a read that depends on
      // the bin map (the partition -- tile_parts -- is sized without it)
      const size_t ct_bytes = 16 + (size_t)d->K * RP * 4;  // [K][RP] (+ alignment)
      const int ct = (QSC_CTILE_CT && (int64_t)R * d->K <= 4 * (int64_t)tb.x &&
                      tshm + ct_bytes <= 160 * 1024) ? 1 : 0;
      if (ct) tshm += ct_bytes;
#define CPASS_TILE_LAUNCH(RPV, ET, KD, LG)                                                     \
  hipLaunchKernelGGL((cpass_tile_kernel<RPV, ET, KD, LG>), dim3((unsigned)d->ntiles), tb, tshm, \
                     s, (const ET*)c_entries, c_width, c_off, c_kmap, nks, NP, d->PT, lk, E,     \
                     d->nbins, R, d->K, ct, S, C, w.slab, w.cnll, w.cnsq,                      \
                     nsq ? w.snsq : nullptr)
      QSC_DISPATCH_PASS(CPASS_TILE_LAUNCH);
#undef CPASS_TILE_LAUNCH
      QSC_CHECK_LAUNCH();
      return QSC_OK;
    }
  }
  if (shm > 160 * 1024) return QSC_EINVAL;
  const int xcd_map = (d->ntiles % 8) == 0 ? 1 : 0;
  const dim3 grid((unsigned)((int64_t)d->ntiles * d->nks));
#define CPASS_LAUNCH(RPV, ET, KD, LG)                                                          \
  hipLaunchKernelGGL((cpass_kernel<RPV, ET, KD, LG>), grid, dim3(kCBlock), shm, s,           \
                     (const ET*)c_entries, c_width, c_off, c_kmap, d->nks, d->PT, xcd_map, lk, \
                     E, d->nbins, R, d->K, S, C, w.slab, w.cnll, w.cnsq)
  QSC_DISPATCH_PASS(CPASS_LAUNCH);
#undef CPASS_LAUNCH
  QSC_CHECK_LAUNCH();
  if (nsq) return qsc_slice_nsq(d, R, S, ws, ws_bytes, stream);  // (per-slice form: unfused)
  return QSC_OK;
}

// fused S-step + next C-pass: the partition (parts per bin list) of the C-pass form qsc_cpass
// uses for this layout -- the tile form's NP, or kCParts where qsc_cpass falls back to the
// per-(tile, k-slice) form -- so that the fused launch sums every dC in the same order
static int cpass_parts(const qsc_obs_desc* d, int R, bool sr) {
  int NP = 1;
  return tile_parts(d, R, sr, &NP) ? NP : kCParts;
}

// the fused launch applies (its C-pass partition and LDS fit), with or without signed rows
static bool scpass_fits(const qsc_obs_desc* d, int R, bool sr) {
  const int NP = cpass_parts(d, R, sr);
  const int U = d->nks * NP;
  // any unit count: small problems (C2: one 64-bin slice, ~13 entries per bin and tile, so one
  // unit per tile) run their C-pass units on the first waves while the rest wait at the end
  return U >= 1 && U <= QSC_CTILE_MAXW && d->PT <= 4096 &&
         scfused_lds(d->PT, R, d->K, d->nks, NP, sr) <= 160 * 1024;
}

// Signed-row layouts (include/qsc.h rowfmt 1): the one-bit kind, narrow entries whose values
// reach row 2K / 2PT, and every pass form the code-field layout would use still fitting its
// LDS (the S-pass at its resident-block count; the C-pass tile form or, where that does not
// apply, the per-slice form; the fused launch where it applies)
static bool sr_layout_ok(const qsc_obs_desc* d, int R) {
  if (d->wide || d->nbins != 2 || (int64_t)sr_rows(d->K) > 0x10000 ||
      (int64_t)sr_rows(d->PT) > 0x10000)
    return false;
  const int RP = rp_of(R);
  if (spass_lds(d, R, true) * spass_bpc(RP) > 160 * 1024) return false;
  int np0 = 1, np1 = 1;
  const bool tile = tile_parts(d, R, false, &np0);
  if (tile ? !tile_parts(d, R, true, &np1) : cpass_lds(d, R, true) > 160 * 1024) return false;
  if (scpass_fits(d, R, false) && !scpass_fits(d, R, true)) return false;
  return true;
}

// a launch's layout / likelihood-kind pairing: signed rows need the one-bit kind
static bool rowfmt_ok(const qsc_obs_desc* d, int R, int kind) {
  if (d->rowfmt == 0) return true;
  return d->rowfmt == 1 && kind == LIK_ONEBIT && sr_layout_ok(d, R);
}

QSC_API int qsc_obs_signed_rows_ok(const qsc_obs_desc* d, int32_t R, const qsc_model* m) {
  if (!desc_ok(d) || !m || R < 1 || R > QSC_MAX_R || m->nbounds - 1 != d->nbins) return 0;
  return (lik_kind(m) == LIK_ONEBIT && sr_layout_ok(d, R)) ? 1 : 0;
}

QSC_API int qsc_scpass_supported(const qsc_obs_desc* d, int32_t R) {
  if (!desc_ok(d) || R < 1 || R > 16) return 0;
  return scpass_fits(d, R, d->rowfmt == 1) ? 1 : 0;
}

// threads of the fused launch at rank R (waves: two S-step slices each, 4..16; 4..8 at rank 16;
// one slice each on tiles of at most QSC_FUSED_ONE_SLICE slices)
#ifndef QSC_FUSED_ONE_SLICE
#define QSC_FUSED_ONE_SLICE 16  // C2 (8-slice tiles, 8 waves): 133 k -> 145 k grad-steps/s
#endif
static unsigned scpass_threads(const qsc_obs_desc* d, int R) {
  const int nsl = d->PT / QSC_SLICE;
  const int per = nsl <= QSC_FUSED_ONE_SLICE ? nsl : nsl / 2;
  return 64u * (unsigned)std::min(rp_of(R) > 8 ? 8 : QSC_FUSED_WAVES, std::max(4, per));
}

QSC_API int qsc_scpass(const qsc_obs_desc* d, const void* s_entries, const int32_t* s_width,
                       const int64_t* s_off, const void* c_entries, const int32_t* c_width,
                       const int64_t* c_off, const int32_t* c_kmap, const qsc_model* m,
                       int32_t R, float* S,
                       const float* C, float* mS, float* vS, const qsc_adam* adam,
                       float lambda_s, qsc_state* st, void* ws, size_t ws_bytes, void* stream) {
  if (!qsc_scpass_supported(d, R) || !m || m->nbounds - 1 != d->nbins || !S || !C || !mS ||
      !vS || !adam || !st || !s_width || !s_off || !c_width || !c_off || !c_kmap ||
      (d->s_entries > 0 && !s_entries) || (d->c_entries > 0 && !c_entries) || !ws ||
      ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  const int RP = rp_of(R);
  const int kind = lik_kind(m);
  const bool sr = d->rowfmt == 1;
  const int NP = cpass_parts(d, R, sr);
  if (!rowfmt_ok(d, R, kind)) return QSC_EINVAL;
  const size_t shm = scfused_lds(d->PT, R, d->K, d->nks, NP, sr);
  PassWs w = carve(d, R, ws);
  Edges E;
  make_edges(m, &E);
  Lik lk = make_lik(m);
  set_dbg(lk, d, sr);
  if (kind == LIK_SQUARED)
    make_sq_targets(m, &E);
  else if (!m->log_model)
    scale_edges(&E, m->nbounds - 1, lk.a);
  const qsc_adam ad = *adam;
  const unsigned threads = scpass_threads(d, R);
  (void)RP;
  hipStream_t s = STREAM(stream);
#define SCPASS_LAUNCH(RPV, ET, KD, LG)                                                         \
  do {                                                                                         \
      hipLaunchKernelGGL((scfused_kernel<RPV, ET, KD, LG>), dim3((unsigned)d->ntiles),         \
                         dim3(threads), shm, s, (const ET*)s_entries, s_width, s_off,         \
                         (const ET*)c_entries, c_width, c_off, c_kmap, d->nks, NP, d->PT, lk, E, \
                         d->nbins, R, d->K, S, C, mS, vS, ad, lambda_s, st, w.snll, w.snsq,    \
                         w.slab, w.cnll, w.cnsq, w.acache);                                    \
  } while (0)
  QSC_DISPATCH_PASS(SCPASS_LAUNCH);
#undef SCPASS_LAUNCH
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}


QSC_API int qsc_cfinish(const qsc_obs_desc* d, int32_t R, float* C, int32_t mode, float* dC,
                        float* mC, float* vC, const qsc_adam* adam, float lambda_c,
                        const float* normsq_c_ext, qsc_state* st, float* hist,
                        int32_t hist_cap, void* ws, size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !C || !st || !ws || ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  if ((mode == 0 || mode == 2) && !dC) return QSC_EINVAL;
  if (mode == 1 && (!mC || !vC || !adam)) return QSC_EINVAL;
  if (mode < 0 || mode > 2) return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  qsc_adam ad{};
  if (adam) ad = *adam;
  hipLaunchKernelGGL(cfinish_kernel, dim3((unsigned)(R * d->nks + 2)), dim3(kFBlock), 0,
                     STREAM(stream), w.slab, d->ntiles, d->nks, R, d->K, C, mode, dC, mC, vC, ad,
                     lambda_c, normsq_c_ext, w.cnsq, st, w.cnll, d->ntiles * d->nks, w.snll,
                     w.snsq, d->Pp / QSC_SLICE, hist, hist_cap, w.acache + 2);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_cupdate(int32_t R, int32_t K, float* C, float* mC, float* vC, const float* g,
                        const qsc_adam* adam, float lambda_c, const float* normsq_s_ext,
                        qsc_state* st, void* stream) {
  if (R < 1 || R > QSC_MAX_R || K < 1 || !C || !mC || !vC || !g || !adam || !st)
    return QSC_EINVAL;
  hipLaunchKernelGGL(cupdate_kernel, dim3(1), dim3(kFBlock), 0, STREAM(stream), R, K, C, mC, vC,
                     g, *adam, lambda_c, normsq_s_ext, st);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_state_flush(const qsc_obs_desc* d, int32_t R, qsc_state* st, float* hist,
                            int32_t hist_cap, void* ws, size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !st || !ws || ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  hipLaunchKernelGGL(flush_kernel, dim3(1), dim3(1024), 0, STREAM(stream), st, w.snll, w.snsq,
                     d->ntiles, d->Pp / QSC_SLICE, hist, hist_cap);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_supdate(const qsc_obs_desc* d, int32_t R, float* S, float* mS, float* vS,
                        const float* g, const qsc_adam* adam, float lambda_s, qsc_state* st,
                        void* ws, size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !S || !mS || !vS || !g || !adam || !st || !ws ||
      ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  const int nslices = d->Pp / QSC_SLICE;
  const dim3 grid((unsigned)ceil_div(nslices, kSWaves)), blk(kSBlock);
  const int RP = rp_of(R);
  hipStream_t hs = STREAM(stream);
  if (RP == 4)
    hipLaunchKernelGGL(supdate_kernel<4>, grid, blk, 0, hs, nslices, S, mS, vS, g, *adam, lambda_s, st, w.snsq);
  else if (RP == 8)
    hipLaunchKernelGGL(supdate_kernel<8>, grid, blk, 0, hs, nslices, S, mS, vS, g, *adam, lambda_s, st, w.snsq);
  else
    hipLaunchKernelGGL(supdate_kernel<16>, grid, blk, 0, hs, nslices, S, mS, vS, g, *adam, lambda_s, st, w.snsq);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_supdate_slices(const qsc_obs_desc* d, int32_t R, int32_t s0, int32_t s1,
                               float* S, float* mS, float* vS, const float* g_own,
                               const qsc_adam* adam, float lambda_s, qsc_state* st, void* ws,
                               size_t ws_bytes, void* stream) {
  const int nslices = d ? d->Pp / QSC_SLICE : 0;
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !S || !mS || !vS || !g_own || !adam || !st ||
      !ws || ws_bytes < ws_bytes_for(d, R) || s0 < 0 || s1 < s0 || s1 > nslices)
    return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  const int n = s1 - s0;
  const dim3 grid((unsigned)std::max<int64_t>(1, ceil_div(n, kSWaves))), blk(kSBlock);
  const int RP = rp_of(R);
  hipStream_t hs = STREAM(stream);
  // (an empty shard still launches one block: it raises the pending S-update flag like the rest)
  if (RP == 4)
    hipLaunchKernelGGL(supdate_slices_kernel<4>, grid, blk, 0, hs, s0, s1, S, mS, vS, g_own, *adam, lambda_s, st, w.snsq);
  else if (RP == 8)
    hipLaunchKernelGGL(supdate_slices_kernel<8>, grid, blk, 0, hs, s0, s1, S, mS, vS, g_own, *adam, lambda_s, st, w.snsq);
  else
    hipLaunchKernelGGL(supdate_slices_kernel<16>, grid, blk, 0, hs, s0, s1, S, mS, vS, g_own, *adam, lambda_s, st, w.snsq);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_slice_nsq(const qsc_obs_desc* d, int32_t R, const float* S, void* ws,
                          size_t ws_bytes, void* stream) {
  if (!desc_ok(d) || R < 1 || R > QSC_MAX_R || !S || !ws || ws_bytes < ws_bytes_for(d, R))
    return QSC_EINVAL;
  PassWs w = carve(d, R, ws);
  const int nslices = d->Pp / QSC_SLICE;
  const dim3 grid((unsigned)ceil_div(nslices, kSWaves)), blk(kSBlock);
  const int RP = rp_of(R);
  hipStream_t hs = STREAM(stream);
  if (RP == 4)
    hipLaunchKernelGGL(slice_nsq_kernel<4>, grid, blk, 0, hs, nslices, S, w.snsq);
  else if (RP == 8)
    hipLaunchKernelGGL(slice_nsq_kernel<8>, grid, blk, 0, hs, nslices, S, w.snsq);
  else
    hipLaunchKernelGGL(slice_nsq_kernel<16>, grid, blk, 0, hs, nslices, S, w.snsq);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_adam_flat(float* p, float* m, float* v, const float* g, int64_t n,
                          const qsc_adam* adam, const qsc_state* st, void* stream) {
  if (n < 0 || !adam || !st || (n > 0 && (!p || !m || !v || !g))) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  const int64_t blocks = std::min<int64_t>(ceil_div(n, 256), (int64_t)cu_count() * 8);
  hipLaunchKernelGGL(adam_flat_kernel, dim3((unsigned)blocks), dim3(256), 0, STREAM(stream), p,
                     m, v, g, n, *adam, st);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

QSC_API int qsc_sumsq_small(const float* x, int32_t n, float* out, void* stream) {
  if (n < 0 || !x || !out) return QSC_EINVAL;
  hipLaunchKernelGGL(sumsq_small_kernel, dim3(1), dim3(1024), 0, STREAM(stream), x, n, out);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

#if QSC_DIAG_STAMPS
QSC_API int qsc_diag_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps),
                                  sizeof(unsigned long long) * (size_t)std::min(n, kStampWaves * kStamps));
}
#endif

QSC_API int qsc_debug_status(int32_t clear) {
#if QSC_DEBUG
  int line = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(&line, HIP_SYMBOL(g_qsc_dbg_line), sizeof(int)) != hipSuccess) return -2;
  if (clear && line) {
    const int zero = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_qsc_dbg_line), &zero, sizeof(int)) != hipSuccess) return -2;
  }
  return line;
#else
  (void)clear;
  return -1;
#endif
}

QSC_API int qsc_selftest_erf(const float* x, int32_t n, float* out, void* stream) {
  if (n < 0 || !x || !out) return QSC_EINVAL;
  if (n == 0) return QSC_OK;
  hipLaunchKernelGGL(selftest_erf_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                     STREAM(stream), x, n, out);
  QSC_CHECK_LAUNCH();
  return QSC_OK;
}

}  // extern "C"
