// qsc_sched.cuh — bank-conflict-free order of the packed observation lists (host + device).
//
// The fused passes gather one LDS row per observed entry (qsc_pass.hip pair_rows): the C-pass
// reads S-tile rows indexed by pixel position, the S-step C^T rows indexed by frequency bin.
// A wave64 ds_read_b128 is serviced as four 16-lane groups, one LDS cycle per group when the
// group's 16 addresses fall in 16 distinct 16-byte bank groups (MI355X_MICROARCH.md, LDS table:
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32).  Every gather table has a row
// pitch of an odd number of 16-byte units (or exactly one), so a row's bank group is a
// bijection of its row index mod 16: a group is conflict-free iff its 16 lanes read rows of 16
// distinct residues mod 16.  With the natural (ascending) list order the residues are random,
// ~3.5 cycles per group instead of 1 (profiles/r02 SQ counters: bank-conflict cycles = 0.65 of
// LDS-index cycles).
//
// The order of the entries inside a lane's list is free (it only changes the summation order
// of the lane's gradient, within the fp32 tolerance), and so is the row an unused (pad) slot
// reads.  For one 16-lane group with lists padded to W slots, slot j of every lane is read by
// the same instruction, so choosing the order is an edge colouring of the bipartite multigraph
// lanes x residues (an entry = an edge, a slot = a colour) with W colours.  A residue with more
// than W entries in the group is split into ceil(count / W) vertices of degree <= W (the first
// W entries to the first, and so on), so every vertex has degree <= W and Koenig's theorem gives
// a W-colouring, with the residue doubled in only count - W slots:
// each slot holds each residue at most ceil(count / W) times (1 whenever count <= W).  The
// colouring is built edge by edge with the classical alternating-path recolouring: for edge
// (u, v) take a colour a free at u and b free at v; if a is not free at v, flip the a/b path
// that starts at v (it cannot reach u in a bipartite graph) and colour the edge a.  Pads then
// take residues no real entry of their slot uses (16 lanes, so there are always enough).
#pragma once
#include <stdint.h>

namespace qsc {

constexpr int kSchedLanes = 16;
constexpr int kSchedMaxV = 48;    // 16 lanes + at most 32 residue vertices (sum ceil(c_r / W))
constexpr int kSchedMaxW = 256;   // longer lists keep their natural order

// i-th lane (i < 16) of ds_read_b128 lane group g (g < 4; groups 0, 1 lie in lanes 0..31)
__host__ __device__ __forceinline__ int b128_group_lane(int g, int i) {
  const int base = (g >> 1) * 32;
  if ((g & 1) == 0) return base + (i < 4 ? i : (i < 8 ? 8 + i : 12 + i));  // 0-3, 12-15, 20-27
  return base + (i < 8 ? 4 + i : (i < 12 ? 8 + i : 16 + i));               // 4-11, 16-19, 28-31
}

__host__ __device__ __forceinline__ int sched_words(int W) { return (W + 31) >> 5; }

// scratch of one group of lists of W slots: at[V][W] (edge id + 1 at (vertex, colour), 0 = free),
// fm[V][words] (free-colour bit masks), ev[16][W] (vertex of the residue side of each edge),
// path[V] (the alternating path being flipped)
__host__ __device__ __forceinline__ size_t sched_scratch_bytes(int W) {
  const size_t b = (size_t)kSchedMaxV * W * 2 + (size_t)kSchedMaxV * sched_words(W) * 4 +
                   (size_t)kSchedLanes * W + (size_t)kSchedMaxV * 2;
  return (b + 15) & ~(size_t)15;
}

struct SchedView {
  uint32_t* fm;
  uint16_t* at;
  uint16_t* path;
  uint8_t* ev;
  int W, words;
};

__host__ __device__ __forceinline__ SchedView sched_view(void* scratch, int W) {
  SchedView v;
  v.W = W;
  v.words = sched_words(W);
  char* p = (char*)scratch;
  v.fm = (uint32_t*)p;
  p += (size_t)kSchedMaxV * v.words * 4;
  v.at = (uint16_t*)p;
  p += (size_t)kSchedMaxV * W * 2;
  v.path = (uint16_t*)p;
  p += (size_t)kSchedMaxV * 2;
  v.ev = (uint8_t*)p;
  return v;
}

__host__ __device__ __forceinline__ int sched_ctz(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_ctz(x);
#else
  return __builtin_ctz(x);
#endif
}

// Entry conventions of one list format (include/qsc.h): residue = row index mod 16 (both the
// code-field and the signed-row values carry the row index in their low bits, and signed rows
// offset the negated half by a multiple of 16), pads recognised and made by value.
struct SchedFmt {
  uint32_t pad_base;  // signed rows: 2 * sr_off (pad rows pad_base + r); code-field: kPad << bits
  uint32_t rows;      // table rows of the index (K or PT): code-field pads must stay below it
  int sr;             // 1: signed-row values, 0: code-field values
  int bits;           // code-field: index bits (12 or 24)

  __host__ __device__ __forceinline__ bool is_pad(uint32_t e) const {
    return sr ? e >= pad_base : (e >> bits) == (pad_base >> bits);
  }
  __host__ __device__ __forceinline__ uint32_t pad(int r) const {
    if (sr) return pad_base + (uint32_t)r;
    return pad_base | ((uint32_t)r < rows ? (uint32_t)r : 0u);
  }
};

__host__ __device__ __forceinline__ int sched_first_free(const SchedView& s, int x) {
  const uint32_t* m = s.fm + x * s.words;
  for (int w = 0; w < s.words; ++w)
    if (m[w]) return (w << 5) + sched_ctz(m[w]);
  return -1;  // unreachable: every vertex has degree <= W
}
__host__ __device__ __forceinline__ bool sched_free(const SchedView& s, int x, int c) {
  return (s.fm[x * s.words + (c >> 5)] >> (c & 31)) & 1u;
}
__host__ __device__ __forceinline__ void sched_take(const SchedView& s, int x, int c, int id) {
  s.at[x * s.W + c] = (uint16_t)(id + 1);
  s.fm[x * s.words + (c >> 5)] &= ~(1u << (c & 31));
}
__host__ __device__ __forceinline__ void sched_drop(const SchedView& s, int x, int c) {
  s.at[x * s.W + c] = 0;
  s.fm[x * s.words + (c >> 5)] |= 1u << (c & 31);
}

// Re-order the lists of one 16-lane group.  Lane i's slot j (natural order) is read with
// get(i, j); the scheduled value of slot c is written with put(i, c, value).  Returns false (and
// writes nothing) if the group cannot be scheduled in this scratch (W > kSchedMaxW or more than
// 65535 entries), so the caller keeps the natural order.
template <class Get, class Put>
__host__ __device__ bool sched_group(void* scratch, int W, const SchedFmt& f, const Get& get,
                                     const Put& put) {
  if (W <= 0 || W > kSchedMaxW || kSchedLanes * W > 65535) return false;
  const SchedView s = sched_view(scratch, W);
  int cnt[16], mult[16], base[16], dealt[16];
  for (int r = 0; r < 16; ++r) cnt[r] = dealt[r] = 0;
  for (int i = 0; i < kSchedLanes; ++i)
    for (int j = 0; j < W; ++j) {
      const uint32_t e = get(i, j);
      if (!f.is_pad(e)) ++cnt[e & 15u];
    }
  int V = kSchedLanes;
  for (int r = 0; r < 16; ++r) {
    mult[r] = cnt[r] > W ? (cnt[r] + W - 1) / W : 1;
    base[r] = V;
    V += mult[r];
  }
  if (V > kSchedMaxV) return false;  // cannot happen: sum ceil(c_r / W) <= 16 + 16
  const uint32_t tail = (W & 31) ? ((1u << (W & 31)) - 1u) : 0xFFFFFFFFu;
  for (int x = 0; x < V; ++x) {
    for (int w = 0; w < s.words; ++w) s.fm[x * s.words + w] = (w == s.words - 1) ? tail : 0xFFFFFFFFu;
    for (int c = 0; c < W; ++c) s.at[x * W + c] = 0;
  }
  for (int i = 0; i < kSchedLanes; ++i)
    for (int j = 0; j < W; ++j) {
      const int id = i * W + j;
      const uint32_t e = get(i, j);
      if (f.is_pad(e)) {
        s.ev[id] = 0xFF;
        continue;
      }
      const int r = (int)(e & 15u);
      // copies filled in turn (W entries each, the last takes the rest): a full copy uses every
      // slot once, so the residue is doubled in exactly count - W slots, the minimum
      const int v = base[r] + dealt[r]++ / W;
      s.ev[id] = (uint8_t)v;
      const int u = i;
      const int a = sched_first_free(s, u);
      const int b = sched_first_free(s, v);
      if (sched_free(s, v, a)) {
        sched_take(s, u, a, id);
        sched_take(s, v, a, id);
        continue;
      }
      if (sched_free(s, u, b)) {
        sched_take(s, u, b, id);
        sched_take(s, v, b, id);
        continue;
      }
      // flip the a/b alternating path that starts at v with its a-edge
      int n = 0, x = v, col = a;
      for (;;) {
        const int e1 = s.at[x * W + col];
        if (!e1) break;
        const int pe = e1 - 1;
        s.path[n++] = (uint16_t)pe;
        const int pl = pe / W;
        x = (x == pl) ? (int)s.ev[pe] : pl;
        col = (col == a) ? b : a;
      }
      for (int k = 0; k < n; ++k) {
        const int pe = s.path[k], oc = (k & 1) ? b : a;
        sched_drop(s, pe / W, oc);
        sched_drop(s, s.ev[pe], oc);
      }
      for (int k = 0; k < n; ++k) {
        const int pe = s.path[k], nc = (k & 1) ? a : b;
        sched_take(s, pe / W, nc, pe);
        sched_take(s, s.ev[pe], nc, pe);
      }
      sched_take(s, u, a, id);
      sched_take(s, v, a, id);
    }
  // slot c of every lane: its coloured entry, or a pad on a residue no entry of slot c reads
  for (int c = 0; c < W; ++c) {
    uint32_t used = 0;
    for (int i = 0; i < kSchedLanes; ++i) {
      const int e1 = s.at[i * W + c];
      if (e1) used |= 1u << (get((e1 - 1) / W, (e1 - 1) % W) & 15u);
    }
    uint32_t freer = ~used & 0xFFFFu;
    for (int i = 0; i < kSchedLanes; ++i) {
      const int e1 = s.at[i * W + c];
      if (e1) {
        put(i, c, get((e1 - 1) / W, (e1 - 1) % W));
      } else {
        const int r = freer ? sched_ctz(freer) : 0;
        freer &= freer - 1u;
        put(i, c, f.pad(r));
      }
    }
  }
  return true;
}

}  // namespace qsc
