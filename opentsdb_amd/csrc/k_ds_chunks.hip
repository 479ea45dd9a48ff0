// k_ds_chunks.hip — streaming greedy downsampling of regular-cadence integer
// spans (the dominant case: series written at a fixed interval), one wave
// per span, emitting E (the span's bucket sequence) directly.
//
// Span.DownsamplingIterator (Span.java:377-422) chains buckets serially: a
// bucket starts at the first point >= previous start + interval. For a span
// whose second bucket starts at cell kk and whose cadence is regular, the
// heads are exactly cells 0, kk, 2kk, ... The wave assumes that and proves it
// as it goes: head h is exact iff ts[h] >= ts[h-kk] + interval > ts[h-1],
// and the span's last cell must lie inside the last bucket. kk is found as
// the first cell at/after ts[0] + interval (any distance, across chunks and
// rows). Any miss, a float cell, a mixed-width or unaligned row, unsorted
// cells, or a first cell before `start` send the whole span to the serial
// kernels (k_decode_fast, then k_decode.hip), which rewrite its E.
//
// The row streams through in 512-cell chunks (8 consecutive cells per lane:
// one 16-B qualifier load and two or four 16-B value loads), the next chunk's
// loads in flight while one is processed. Per chunk, DPP wave scans build ts-delta and value prefixes in LDS;
// lane j owns the chunk's j-th head, and a bucket's count / ts sum / integer
// sum are prefix differences (exact in any order). The bucket still open at
// the end of a chunk (or row) is carried in registers and completed by the
// next chunk's lead cells, so every bucket leaves the kernel finished: no
// pieces, no second pass.
//
// Once a span is proven, the wave marks its E timestamps in the union-grid
// bitmap (re-reading the E it just wrote; the span's loads have drained by
// then), which saves the separate k_grid_mark pass for these spans.
//
// The chunk loop issues no global load besides the chunk stream itself: an
// in-order vmcnt wait for any other load would also drain the prefetched
// chunks.
#pragma once
#include "dev_common.h"
#include "k_decode_fast.hip"

namespace tsdb {

struct SpanDsArgs {
  uint32_t* list;        // spans left to the serial kernels
  uint32_t* list_count;  // [1], or [nseg]
  // nseg > 0: `list` is nseg segments of seg_cap entries, block b appending
  // to segment b % nseg with its own counter (one wave per span appends
  // once per rejected span: one shared counter would serialise 10k+
  // same-address atomics when whole groups are rejected, e.g. float spans
  // passing through the integer instantiation)
  uint32_t nseg, seg_cap;
  const uint32_t* in_list;   // spans to take (null: every kept span)
  const uint32_t* in_count;  // [1], or [in_nseg]
  uint32_t in_nseg, in_seg_cap;
  uint32_t* bitmap;      // union-grid bitmap over [lo, hi] (null: no marking)
  int64_t lo, hi;
  int32_t rate;
};

constexpr uint32_t DCH = 512;  // cells per chunk: 8 per lane

template <int W>
struct RawW {
  uint4 q;              // 8 big-endian qualifiers
  uint4 v[2 * W / 4];   // 8 values
};

// Branch-free chunk load of 8 consecutive cells per lane; c is clamped into
// the row by the caller. Reads up to 7 cells past the row end (inside the
// buffers' 64-byte slack). Lanes read 16 B of qualifiers and 8W bytes of
// values each (plain loads: non-temporal ones measured 15 % slower).
template <int W>
DEVI void load_raw(const DecodeArgs& a, uint64_t qoff, uint64_t voff, uint32_t c, RawW<W>& x) {
  x.q = *(const uint4*)(a.qual + qoff + 2ull * c);
  const uint4* pv = (const uint4*)(a.val + voff + (uint64_t)W * c);
#pragma unroll
  for (int i = 0; i < 2 * W / 4; i++) x.v[i] = pv[i];
}

template <int W>
DEVI int64_t raw_value(const RawW<W>& x, int j) {
  if (W == 8) {
    const uint4 u = x.v[j >> 1];
    const uint32_t lo = (j & 1) ? u.z : u.x, hi = (j & 1) ? u.w : u.y;
    return (int64_t)bswap64((uint64_t)lo | ((uint64_t)hi << 32));
  }
  const uint4 u = x.v[j >> 2];
  const int k = j & 3;
  const uint32_t w = k == 0 ? u.x : k == 1 ? u.y : k == 2 ? u.z : u.w;
  return (int64_t)(int32_t)bswap32(w);
}

// Two big-endian qualifiers of one dword -> (q0 | q1 << 16) in native order.
DEVI uint32_t qpair(uint32_t word) { return __builtin_amdgcn_perm(word, word, 0x02030001u); }

// Open-bucket / chain state of one span (wave-uniform).
struct DsState {
  uint32_t kk;       // cells per bucket (0 until the second head is found)
  uint32_t hnext;    // span cell index of the next head (~0u: not in sight)
  uint32_t bnext;    // bucket index of hnext
  uint32_t t0;       // ts of the span's first cell
  uint32_t lh_ts;    // ts of the latest head
  uint32_t prev_ts;  // ts of the latest cell
  bool open;         // bucket bnext-1 still takes cells
  uint32_t o_n;      // its cells so far
  uint64_t o_rel;    // its sum of (ts - o_ref)
  uint32_t o_ref;    // its head ts
  int64_t o_v;       // its value sum / min / max
  uint32_t fbase;    // first bucket index held in the LDS buffer
  uint32_t room;     // most buckets one chunk can close (256 / kk + 2)
};

// Closed buckets wait in a per-wave LDS buffer (count, ts offsets, value)
// and leave it in batches, one lane per bucket, so the divisions of
// Span.java:399 and the avg downsampler stay out of the chunk loop. A chunk
// closes at most 512/kk + 2 <= 130 buckets (kk >= 4).
constexpr uint32_t BKB = 136;
struct BkLds {
  uint32_t ref[BKB];  // head ts
  uint32_t n[BKB];    // cells
  uint64_t rel[BKB];  // sum of (ts - ref)
  int64_t v[BKB];     // value sum / min / max
};

// Scalar (SMEM) load of read-only metadata at a wave-uniform address: the
// span prologue's dependent chain (kept -> span rows -> row fields) then waits
// on lgkmcnt through the scalar cache instead of one vmcnt(0) round trip per
// level. Only for arrays no kernel in flight writes.
template <class T>
DEVI T sld(const T* p) { return *(const __attribute__((address_space(4))) T*)p; }
// the byte at p through the aligned dword holding it
DEVI uint32_t sld_u8(const uint8_t* p) {
  const uintptr_t u = (uintptr_t)p;
  return (sld((const uint32_t*)(u & ~(uintptr_t)3)) >> (8 * (u & 3))) & 0xFFu;
}

// wave-uniform copies (SGPR) of values every lane holds alike
DEVI uint32_t ufl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEVI uint64_t ufl64(uint64_t x) { return ((uint64_t)ufl((uint32_t)(x >> 32)) << 32) | (uint64_t)ufl((uint32_t)x); }

// Writes buckets [b0, b0 + cnt) of the span to E (Span.java:396-420, integer
// buckets); returns each lane's bucket ts (lane < cnt).
template <int AGG>
DEVI uint32_t bk_flush(const DecodeArgs& a, const BkLds& B, uint64_t eo, uint32_t cap, uint32_t b0, uint32_t cnt,
                       bool flt, bool& bad) {
  wave_lds_sync();
  const int lane = lane_id();
  uint32_t ts0 = 0;
  for (uint32_t i = lane; i < cnt; i += WAVE) {
    const uint32_t b = b0 + i;
    const uint32_t n = B.n[i];
    const uint32_t ts = B.ref[i] + (uint32_t)udiv64_32(B.rel[i], n);  // Span.java:399
    if (i == (uint32_t)lane) ts0 = ts;
    if (b < cap) {
      a.e_ts[eo + b] = ts;
      if (flt)  // Aggregators.Avg.runDouble: sum / n (Aggregators.java:172-180)
        a.e_val[eo + b] = AGG == 3 ? dbits(bitsd(B.v[i]) / (double)(int32_t)n) : B.v[i];
      else
        a.e_val[eo + b] = AGG == 3 ? ldiv64_32(B.v[i], n) : B.v[i];
      a.e_flt[eo + b] = flt ? 1 : 0;
    } else {
      bad = true;  // more buckets than E holds: cannot be the greedy chain
    }
  }
  wave_lds_sync();
  return ts0;
}

// runDouble of sum / min / max / avg, one value at a time in point order,
// seeded with the first (Aggregators.java:86-180)
template <int AGG>
DEVI double ds_dcombine(double x, double y) {
  if (AGG == 0 || AGG == 3) return x + y;
  if (AGG == 1) return y < x ? y : x;
  return y > x ? y : x;
}

template <int AGG>
DEVI int64_t ds_combine(int64_t x, int64_t y) {
  if (AGG == 0 || AGG == 3) return ladd(x, y);
  if (AGG == 1) return y < x ? y : x;
  return y > x ? y : x;
}

// Position of one chunk in a span's row sequence (wave-uniform): the row's
// fields, the span cell index of the row's first cell, the chunk's first
// cell in the row. `done`: past the span's last chunk.
struct ChunkPos {
  uint64_t qoff, voff, r;
  uint32_t base, nc, cell0, c0;
  bool done;
};

// A span's 512-cell chunks, row after row, as one stream: two register sets,
// the next chunk's loads (in this row or the next one) in flight while one
// is processed, so a span of short rows (C2: 360 cells per row) does not wait
// one full load latency per row. Rows [r0, r1) were checked by the caller
// (row_ok, cells, width W, alignment). Returns true if a precondition breaks
// (the span then goes to the serial path).
template <int AGG, int W, bool FLT>
DEVI bool ds_span(const DecodeArgs& a, DsState& st, uint64_t eo, uint32_t cap, uint64_t r0, uint64_t r1,
                  const uint32_t* ncells, uint32_t* L_pt, uint64_t* L_v, BkLds& BK) {
  constexpr bool PREFIX = AGG == 0 || AGG == 3;  // sum / avg: prefix differences; min / max: loops
  const int lane = lane_id();
  const int64_t I = a.interval;
  // ts delta (from the row base) of chunk cell x: the ts prefix differenced
  auto dtx = [&](uint32_t x) { return L_pt[x] - (x > 0 ? L_pt[x - 1] : 0u); };
  auto row_at = [&](uint64_t r, uint32_t cell0) {
    ChunkPos p;
    p.r = r;
    p.nc = sld(&ncells[r]);
    p.qoff = sld(&a.row_qual_off[r]);
    p.voff = sld(&a.row_val_off[r]);
    p.base = sld(&a.row_base[r]);
    p.cell0 = cell0;
    p.c0 = 0;
    p.done = false;
    return p;
  };
  auto advance = [&](const ChunkPos& p) {
    if (p.done) return p;
    if (p.c0 + DCH < p.nc) {
      ChunkPos q = p;
      q.c0 += DCH;
      return q;
    }
    if (p.r + 1 < r1) return row_at(p.r + 1, p.cell0 + p.nc);
    ChunkPos q = p;
    q.done = true;
    return q;
  };
  RawW<W> A, B;
  // (a done position re-loads its own cells: branch-free, cache hits)
  auto issue = [&](const ChunkPos& p, RawW<W>& x) {
    const uint32_t c = p.c0 + 8u * lane;
    __builtin_amdgcn_s_setprio(2);  // the chunk's loads ahead of other waves' VALU
    load_raw<W>(a, p.qoff, p.voff, c < p.nc ? c : (p.nc - 1) & ~7u, x);
    __builtin_amdgcn_s_setprio(0);
  };
  bool bad = false;
  auto step = [&](const ChunkPos& p, const RawW<W>& cur) {
    const uint32_t c0 = p.c0, nc = p.nc, base = p.base, cell0 = p.cell0;
    const uint32_t nv = min(DCH, nc - c0);
    const uint32_t cs = cell0 + c0;  // span cell index of the chunk start
    // ---- decode: 8 cells per lane (loads past the row end were clamped) ----
    uint32_t qp[4];
    qp[0] = qpair(cur.q.x);
    qp[1] = qpair(cur.q.y);
    qp[2] = qpair(cur.q.z);
    qp[3] = qpair(cur.q.w);
    constexpr bool prefix = PREFIX && !FLT;
    uint32_t dt[8];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      dt[2 * i] = (qp[i] & 0xFFFF) >> 4;
      dt[2 * i + 1] = qp[i] >> 20;
    }
    int64_t bits[8];
#pragma unroll
    for (int j = 0; j < 8; j++) bits[j] = raw_value<W>(cur, j);
    if (W == 4 && FLT) {  // float32 cells widened to double (RowSeq.java:216-226)
#pragma unroll
      for (int j = 0; j < 8; j++) bits[j] = dbits((double)__int_as_float((int32_t)bits[j]));
    }
    // integer cells of width W (flags nibble of each qualifier), strictly
    // increasing deltas (Span/RowSeq order)
    const uint32_t fl = ((FLT ? 8u : 0u) | (W - 1)) * 0x00010001u;
    uint32_t nmine = 8;
    if (nv == DCH) {  // full chunk: every lane holds 8 cells
      bad |= (((qp[0] ^ fl) | (qp[1] ^ fl) | (qp[2] ^ fl) | (qp[3] ^ fl)) & 0x000F000Fu) != 0;
#pragma unroll
      for (int j = 1; j < 8; j++) bad |= dt[j] <= dt[j - 1];
    } else {  // the row's last chunk: mask the lanes past its end
      nmine = nv > 8u * lane ? min(8u, nv - 8u * lane) : 0u;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t fm = nmine >= 2u * i + 2 ? 0x000F000Fu : (nmine == 2u * i + 1 ? 0x0000000Fu : 0u);
        bad |= ((qp[i] ^ fl) & fm) != 0;
      }
#pragma unroll
      for (int j = 1; j < 8; j++) bad |= (uint32_t)j < nmine && dt[j] <= dt[j - 1];
      if (nmine == 0) dt[0] = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if (j > 0 && (uint32_t)j >= nmine) dt[j] = dt[j - 1];  // ts prefix flat past the end
        if ((uint32_t)j >= nmine) bits[j] = 0;
      }
    }
    {
      const uint32_t pl = shfl_up_u32(dt[7], 1);
      bad |= lane > 0 && nmine > 0 && dt[0] <= pl;
      bad |= lane == 0 && cs > 0 && base + dt[0] <= st.prev_ts;  // previous chunk / row
    }
    // ---- stage: ts prefix, value prefix (or raw values) ----
    uint32_t pt = 0;
    uint64_t pv = 0;
    uint32_t pti[8];
    uint64_t pvi[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      pt += (uint32_t)j < nmine ? dt[j] : 0u;  // (nmine == 8 on full chunks)
      pv += (uint64_t)bits[j];
      pti[j] = pt;
      pvi[j] = prefix ? pv : (uint64_t)bits[j];
    }
    const uint32_t xt = wave_incl_scan_u32_dpp(pt) - pt;
    *(uint4*)&L_pt[8 * lane] = make_uint4(pti[0] + xt, pti[1] + xt, pti[2] + xt, pti[3] + xt);
    *(uint4*)&L_pt[8 * lane + 4] = make_uint4(pti[4] + xt, pti[5] + xt, pti[6] + xt, pti[7] + xt);
    {
      const uint64_t xv = prefix ? wave_incl_scan_u64_dpp(pv) - pv : 0ull;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        ulonglong2 v2;
        v2.x = pvi[j] + xv;
        v2.y = pvi[j + 1] + xv;
        *(ulonglong2*)&L_v[8 * lane + j] = v2;
      }
    }
    wave_lds_sync();
    const uint32_t cend = cs + nv;
    // ---- the span's first cell opens bucket 0 ----
    if (cs == 0) {
      st.t0 = ufl(base + L_pt[0]);
      bad |= (int64_t)st.t0 < a.start;  // no seek inside the span
      st.lh_ts = st.t0;
      st.open = true;
      st.o_n = 0;
      st.o_rel = 0;
      st.o_ref = st.t0;
      st.o_v = AGG == 1 ? INT64_MAX : (AGG == 2 ? INT64_MIN : 0);
      st.bnext = 1;
      st.hnext = ~0u;
      st.fbase = 0;
    }
    // ---- second head: the first cell at/after t0 + interval ----
    if (st.kk == 0) {
      const int64_t end0 = (int64_t)st.t0 + I;
      uint64_t m = 0;
      int q = 0;
      for (; q < (int)(DCH / WAVE) && !m; q++) {
        const uint32_t c = 64u * q + lane;
        m = ballot(c < nv && (int64_t)(base + L_pt[c] - (c > 0 ? L_pt[c - 1] : 0u)) >= end0);
      }
      if (m) {
        st.kk = cs + 64u * (q - 1) + (uint32_t)(__ffsll((long long)m) - 1);
        st.hnext = st.kk;
        st.room = DCH / max(st.kk, 4u) + 2;
        bad |= st.kk < 4;  // more than 128 heads per chunk: the serial kernels
      }
    }
    // ---- room in the bucket buffer for every bucket this chunk can close ----
    if (st.kk != 0) {
      const uint32_t closed = st.bnext - (st.open ? 1u : 0u);
      if (closed + st.room - st.fbase > BKB) {
        bk_flush<AGG>(a, BK, eo, cap, st.fbase, closed - st.fbase, FLT, bad);
        st.fbase = closed;
      }
    }
    // ---- lead cells [cs, min(hnext, cend)) complete the open bucket ----
    const uint32_t lend = min(st.hnext, cend);
    if (lend > cs) {
      const uint32_t ln = lend - cs;
      bad |= !st.open;
      const bool seed = st.o_n == 0;
      st.o_n += ln;
      st.o_rel += (uint64_t)ln * base + ufl(L_pt[ln - 1]) - (uint64_t)ln * st.o_ref;
      if (prefix) {
        st.o_v = ladd(st.o_v, (int64_t)ufl64(L_v[ln - 1]));
      } else if (FLT) {  // the open double bucket continues in point order
        double v = bitsd(st.o_v);
        for (uint32_t i = 0; i < ln; i++) {
          const double x = bitsd((int64_t)L_v[i]);
          v = (seed && i == 0) ? x : ds_dcombine<AGG>(v, x);
        }
        st.o_v = dbits(v);
      } else {
        int64_t v = AGG == 1 ? INT64_MAX : INT64_MIN;
        for (uint32_t i = lane; i < ln; i += WAVE) v = ds_combine<AGG>(v, (int64_t)L_v[i]);
        v = AGG == 1 ? wave_min_i64(v) : wave_max_i64(v);
        st.o_v = ds_combine<AGG>(st.o_v, (int64_t)ufl64((uint64_t)v));
      }
    }
    // ---- heads hnext, hnext + kk, ... inside the chunk ----
    if (st.hnext < cend) {
      const uint32_t kk = st.kk;
      {  // the first head closes the open bucket: prove it against the latest head
        const uint32_t la = st.hnext - cs;
        const int64_t th = ufl(base + dtx(la));
        const int64_t tp = la > 0 ? (int64_t)ufl(base + dtx(la - 1)) : (int64_t)st.prev_ts;
        const int64_t e = (int64_t)st.lh_ts + I;
        bad |= !(th >= e && tp < e);
        if (st.open) {
          const uint32_t b = st.bnext - 1;
          if (lane == 0) {
            const uint32_t sl = b - st.fbase;
            BK.ref[sl] = st.o_ref;
            BK.n[sl] = st.o_n;
            BK.rel[sl] = st.o_rel;
            BK.v[sl] = st.o_v;
          }
        }
        st.open = false;
      }
      const uint32_t nh = min((cend - 1 - st.hnext) / max(kk, 4u) + 1, 2u * WAVE);  // kk >= 4
      for (uint32_t jb = 0; jb < nh; jb += WAVE) {
        const uint32_t j = jb + lane;
        const bool mine = j < nh;
        const uint32_t H = st.hnext + j * kk;
        const uint32_t la = mine ? H - cs : 0;
        const uint32_t lb = mine ? min(H + kk, cend) - 1 - cs : 0;
        const uint32_t n = lb - la + 1;
        const uint32_t pa = la > 0 ? L_pt[la - 1] : 0u;
        const uint32_t dta = L_pt[la] - pa;
        const uint32_t ref = base + dta;
        const uint32_t rel = (L_pt[lb] - pa) - n * dta;
        int64_t v;
        if (prefix) {
          v = (int64_t)(L_v[lb] - (la > 0 ? L_v[la - 1] : 0ull));
        } else if (FLT) {
          double d = bitsd((int64_t)L_v[la]);
          for (uint32_t i = la + 1; i <= lb; i++) d = ds_dcombine<AGG>(d, bitsd((int64_t)L_v[i]));
          v = dbits(d);
        } else {
          v = (int64_t)L_v[la];
          for (uint32_t i = la + 1; i <= lb; i++) v = ds_combine<AGG>(v, (int64_t)L_v[i]);
        }
        if (mine && j > 0) {  // chain proof against the previous head of the chunk
          const uint32_t tprev = base + dtx(la - kk);
          const uint64_t e64 = (uint64_t)tprev + (uint64_t)I;
          const uint32_t e = (uint32_t)e64;
          bad |= e64 > 0xFFFFFFFFull ? true : !(ref >= e && base + (pa - (la > 1 ? L_pt[la - 2] : 0u)) < e);
        }
        // closed buckets st.bnext + j (complete inside the chunk) -> LDS buffer
        if (mine && H + kk <= cend) {
          const uint32_t sl = st.bnext + j - st.fbase;
          BK.ref[sl] = ref;
          BK.n[sl] = n;
          BK.rel[sl] = rel;
          BK.v[sl] = v;
        }
        if (jb + WAVE >= nh) {  // the chunk's last head: latest head, maybe still open
          const int l = (int)(nh - 1 - jb);
          st.lh_ts = readlane_u32(ref, l);
          const uint32_t Hl = st.hnext + (nh - 1) * kk;
          if (Hl + kk > cend) {
            st.open = true;
            st.o_n = readlane_u32(n, l);
            st.o_rel = readlane_u32(rel, l);
            st.o_ref = st.lh_ts;
            st.o_v = (int64_t)readlane_u64((uint64_t)v, l);
          }
        }
      }
      st.hnext += nh * kk;
      st.bnext += nh;
    }
    st.prev_ts = ufl(base + dtx(nv - 1));
    wave_lds_sync();
  };
  // two register sets: one chunk in flight while the other is processed
  ChunkPos p0 = row_at(r0, 0);
  ChunkPos p1 = advance(p0);
  issue(p0, A);
  issue(p1, B);
  // (a broken precondition ends the stream: the chain state past it is
  // meaningless, and the span is redone by the serial kernels)
  for (;;) {
    step(p0, A);
    if (p1.done || ballot(bad) != 0) break;
    const ChunkPos p2 = advance(p1);
    issue(p2, A);
    step(p1, B);
    if (p2.done || ballot(bad) != 0) break;
    const ChunkPos p3 = advance(p2);
    issue(p3, B);
    p0 = p2;
    p1 = p3;
  }
  return ballot(bad) != 0;
}

// One wave per kept span (or per span of g.in_list). FLTM 0: integer spans,
// 1: float spans (double buckets), 2: either, by the span's first cell (one
// launch for k_ds_reg's few leftovers).
template <int AGG, int FLTM>
__global__ void __launch_bounds__(256) k_ds_spans(DecodeArgs a, SpanDsArgs g, const uint32_t* ncells,
                                                  const uint32_t* vlen) {
  __shared__ uint32_t s_pt[4][DCH];
  __shared__ uint64_t s_v[4][DCH];
  __shared__ BkLds s_bk[4];
  const int lane = lane_id();
  const int wib = threadIdx.x / WAVE;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  bool any_i = false, any_f = false;
  int64_t fs = 0;  // F*: latest first bucket ts of a float span, + 1
  // a segmented input list: segment counts lane-parallel, their exclusive
  // prefix locates item w
  uint32_t seg_ex = 0;
  uint32_t n_in = a.n_kept;
  if (g.in_list && g.in_nseg) {
    const uint32_t c = (uint32_t)lane < g.in_nseg ? g.in_count[lane] : 0u;
    const uint32_t inc = wave_incl_scan_u32_dpp(c);
    seg_ex = inc - c;
    n_in = readlane_u32(inc, 63);
  } else if (g.in_list) {
    n_in = sld(g.in_count);
  }
  for (uint32_t w = ufl(wave); w < n_in; w += nwaves) {
    uint32_t k = w;
    if (g.in_list && g.in_nseg) {
      const uint64_t m = ballot((uint32_t)lane < g.in_nseg && seg_ex <= w);
      const int sg = 63 - __builtin_clzll(m);
      k = sld(&g.in_list[(uint64_t)sg * g.in_seg_cap + (w - readlane_u32(seg_ex, sg))]);
    } else if (g.in_list) {
      k = sld(&g.in_list[w]);
    }
    const uint32_t s = sld(&a.kept[k]);
    const uint64_t r0 = sld(&a.span_row_start[s]), r1 = sld(&a.span_row_start[s + 1]);
    const uint32_t n = sld(&a.sp_ncells[s]);
    bool ok = sld(&a.sp_q1[s]) < 0 && sld(&a.sp_ovf_cell[s]) < 0 && n > 0 && r1 > r0 && a.interval > 0;
    // value width of the span's rows: the first row's, every row must match
    // it and be aligned (checked here, so the chunk stream never stops at a
    // row boundary)
    uint32_t W = 0;
    bool FLT = FLTM == 1;
    if (ok) {
      const uint32_t nc = sld(&ncells[r0]), vl = sld(&vlen[r0]);
      const uint32_t vb = nc > 1 ? vl - 1 : vl;
      W = nc != 0 && vb == (vb / nc) * nc ? vb / nc : 0;
      ok = W == 8 || W == 4;
      // the first cell's type picks the instantiation: the other one leaves
      // the span without streaming it (float spans pass through the integer
      // kernel first)
      if (ok) {
        const bool f0 = (sld_u8(a.qual + sld(&a.row_qual_off[r0]) + 1) & 8u) != 0;
        if (FLTM == 2) FLT = f0;
        ok = f0 == FLT;
      }
    }
    if (ok && r1 - r0 == 1) {  // (one row: the usual hourly span)
      ok = sld_u8(&a.row_ok[r0]) != 0 && (sld(&a.row_qual_off[r0]) & 7) == 0 && (sld(&a.row_val_off[r0]) & 15) == 0;
    } else {
      for (uint64_t rb = r0; ok && rb < r1; rb += WAVE) {  // (uniform loop: keeps `ok` scalar)
        const uint64_t r = rb + lane;
        bool rbad = false;
        if (r < r1) {
          const uint32_t nc = ncells[r], vl = vlen[r];
          const uint32_t vb = nc > 1 ? vl - 1 : vl;
          rbad = a.row_ok[r] == 0 || nc == 0 || vb != W * nc || (a.row_qual_off[r] & 7) != 0 ||
                 (a.row_val_off[r] & 15) != 0;
        }
        ok = ballot(rbad) == 0;
      }
    }
    const uint64_t eo = sld(&a.e_off[k]);
    const uint32_t cap = (uint32_t)sld(&a.sp_cap[s]);
    DsState st = {};
    if (ok) {
      bool fail;
      if (FLTM != 1 && !FLT)
        fail = W == 8 ? ds_span<AGG, 8, false>(a, st, eo, cap, r0, r1, ncells, s_pt[wib], s_v[wib], s_bk[wib])
                      : ds_span<AGG, 4, false>(a, st, eo, cap, r0, r1, ncells, s_pt[wib], s_v[wib], s_bk[wib]);
      else
        fail = W == 8 ? ds_span<AGG, 8, true>(a, st, eo, cap, r0, r1, ncells, s_pt[wib], s_v[wib], s_bk[wib])
                      : ds_span<AGG, 4, true>(a, st, eo, cap, r0, r1, ncells, s_pt[wib], s_v[wib], s_bk[wib]);
      ok = !fail;
    }
    uint32_t ts_last = 0, n_last = 0;  // the final flush (one lane per bucket)
    if (ok) {  // the last cell must lie inside the last bucket; then close it
      bool bad = !((int64_t)st.prev_ts < (int64_t)st.lh_ts + a.interval) || st.bnext > cap;
      const uint32_t b = st.bnext - 1;  // the open bucket
      if (st.open) {
        if (b - st.fbase >= BKB) {  // (cannot happen: a chunk left room for it)
          bk_flush<AGG>(a, s_bk[wib], eo, cap, st.fbase, b - st.fbase, FLT, bad);
          st.fbase = b;
        }
        if (lane == 0) {
          const uint32_t sl = b - st.fbase;
          s_bk[wib].ref[sl] = st.o_ref;
          s_bk[wib].n[sl] = st.o_n;
          s_bk[wib].rel[sl] = st.o_rel;
          s_bk[wib].v[sl] = st.o_v;
        }
      }
      n_last = st.bnext - st.fbase;
      ts_last = bk_flush<AGG>(a, s_bk[wib], eo, cap, st.fbase, n_last, FLT, bad);
      ok = ballot(bad) == 0;
    }
    if (ok) {
      const uint32_t nb = st.bnext;
      if (lane == 0) {
        a.e_len[k] = nb;
        a.e_bad[k] = -1;
      }
      if (FLT) {
        any_f = true;
        if (!a.rate) {  // (the first bucket's ts: lane 0's of the last flush, or E)
          uint32_t t0b;
          if (st.fbase == 0) {
            t0b = readlane_u32(ts_last, 0);
          } else {
            __threadfence_block();
            t0b = ufl(a.e_ts[eo]);
          }
          fs = max(fs, (int64_t)t0b + 1);
        }
      } else {
        any_i = true;
      }
      if (g.bitmap) {  // G: this span's E points <= end (rate: from the second)
        auto mark = [&](int64_t t, uint32_t b) {
          if ((g.rate && b == 0) || t > g.hi || t < g.lo) return;
          const uint64_t off = (uint64_t)(t - g.lo);
          const uint32_t bit = 1u << (off & 31);
          uint32_t* w = &g.bitmap[off >> 5];
          if (!(*w & bit)) atomicOr(w, bit);
        };
        if ((uint32_t)lane < min(n_last, (uint32_t)WAVE)) mark(ts_last, st.fbase + lane);
        if (st.fbase > 0 || n_last > WAVE) {  // buckets not in registers: read their E back
          __threadfence_block();
          for (uint32_t i = lane; i < nb; i += WAVE)
            if (i < st.fbase || i >= st.fbase + WAVE) mark(a.e_ts[eo + i], i);
        }
      }
    } else if (lane == 0) {
      if (g.nseg) {
        const uint32_t sg = blockIdx.x % g.nseg;
        g.list[(uint64_t)sg * g.seg_cap + atomicAdd(&g.list_count[sg], 1u)] = k;
      } else {
        g.list[atomicAdd(g.list_count, 1u)] = k;
      }
    }
  }
  if (lane == 0) {
    if (any_i && !a.gflags[1]) atomicOr(&a.gflags[1], 1u);
    if (any_f && !a.gflags[0]) atomicOr(&a.gflags[0], 1u);
    if (fs && (unsigned long long)fs > *(volatile unsigned long long*)a.fstar)
      atomicMax(a.fstar, (unsigned long long)fs);
  }
}

}  // namespace tsdb
